# PMC passes over the bucket round kernels (scripts/ab_bkt.py, 1M x 1M, 64 nnz, batch 100k): one rocprofv3 run per
# counter set, each under its own KILL timeout; prints per-kernel mean counter values per dispatch.
set -u
root=$(pwd)
mkdir -p gpurun_out/pmc_bkt
export TMPDIR=/tmp
i=0
for set_ in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE" "WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $set_ -d /tmp/pmc_bkt_$i -o run --output-format csv -- python3 $root/scripts/ab_bkt.py 32768) > gpurun_out/pmc_bkt/pass_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/pmc_bkt/pass_$i.log; exit $rc; }
  f=$(find /tmp/pmc_bkt_$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$i" <<'PY'
import csv, sys, collections, json
f, i = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    name = r.get("Kernel_Name", "")
    if "glm_bkt" not in name: continue
    key = "fwd_scatter" if "fwd_scatter" in name else ("bwd" if "bwd" in name else name.split("(")[0][-40:])
    agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: round(sum(v) / len(v), 1) for c, v in d.items()} for k, d in agg.items()}
print(json.dumps({"pass": int(i), "mean_per_dispatch": out}))
PY
done
