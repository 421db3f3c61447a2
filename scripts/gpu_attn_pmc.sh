set -o pipefail
# counters of the attention kernels (fwd, dq, text dK/dV) at B16, axial_row; two passes
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/apmc_$name -o run --output-format csv -- python3 benchmarks/bench_attn_kernel.py axial_row 16 3 > gpurun_out/apmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -20 gpurun_out/apmc_$name.log; exit 1; }
  rm -f gpurun_out/apmc_$name/run_kernel_trace.csv
}
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA
pass b SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS
python3 - <<'PY'
import csv, collections, glob
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/apmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "attn" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    print("   " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
PY
