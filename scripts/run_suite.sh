#!/bin/bash
# Runs the reference benchmark suite on the GPU box: numeric stages at their configured sizes,
# the host-bound string stages (HOST regex) capped at MAX_STRING_VALUES rows (the result keeps
# configuredNumValues). Usage: bash scripts/run_suite.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HOST="(countvectorizer|hashingtf|ngram|regextokenizer|stopwordsremover|stringindexer|tokenizer|sqltransformer)"
timeout -k 10 "${SUITE_TIMEOUT:-900}" python -u -m flink_ml_amd.bench.run flink_ml_amd/bench/conf/reference-suite.json \
  --pattern "^(?!$HOST).*" --warmup "${WARMUP:-1}" --output-file "${OUT:-gpurun_out/suite.json}" > gpurun_out/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 "${SUITE_TIMEOUT:-900}" python -u -m flink_ml_amd.bench.run flink_ml_amd/bench/conf/reference-suite.json \
  --pattern "^$HOST" --max-values "${MAX_STRING_VALUES:-1000000}" --output-file "${OUT_STR:-gpurun_out/suite_strings.json}" > gpurun_out/suite_strings.log 2>&1
rc=$?; echo "string suite rc=$rc"
exit $rc
