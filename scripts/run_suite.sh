#!/bin/bash
# Runs the reference benchmark suite on the GPU box: numeric stages at full size, host/string
# stages listed in HOST_PATTERN separately. Usage: PATTERN=<regex> bash scripts/run_suite.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PATTERN="${PATTERN:-^(?!(countvectorizer|hashingtf|ngram|regextokenizer|stopwordsremover|stringindexer|tokenizer|sqltransformer)).*}"
OUT="${OUT:-gpurun_out/suite.json}"
timeout -k 10 "${SUITE_TIMEOUT:-900}" python -m flink_ml_amd.bench.run flink_ml_amd/bench/conf/reference-suite.json \
  --pattern "$PATTERN" --warmup "${WARMUP:-1}" --output-file "$OUT" > gpurun_out/suite.log 2>&1
rc=$?
echo "suite rc=$rc"
tail -40 gpurun_out/suite.log
exit $rc
