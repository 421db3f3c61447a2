# Round-4 GPU check: every GPU test, smoke, bench (step + collab), a 2-rank gloo rehearsal with the
# reduce-scatter + all-gather path, a kernel trace of the bench step and one PMC pass per counter group.
# usage: bash scripts/gpu_r4_check.sh TAG [quick]
set -o pipefail
TAG=${1:-r4}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_step.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench_step.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_step.log | cut -c1-300
[ "$2" = quick ] && exit 0
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --engine collab > gpurun_out/${TAG}_bench_collab.log 2>&1 || { echo "bench collab failed"; tail -20 gpurun_out/${TAG}_bench_collab.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_collab.log | cut -c1-300
BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 --allreduce-algo rs_ag > gpurun_out/${TAG}_bench_2rank_gloo.log 2>&1 || { echo "2-rank failed"; tail -20 gpurun_out/${TAG}_bench_2rank_gloo.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_2rank_gloo.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
rm -f gpurun_out/prof_${TAG}/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_${TAG}/run_kernel_stats.csv 40 7 > gpurun_out/prof_${TAG}_top.txt
head -25 gpurun_out/prof_${TAG}_top.txt
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc_${TAG}_$name.log 2>&1 || { echo "pmc $name failed"; tail -20 gpurun_out/pmc_${TAG}_$name.log; exit 1; }
  rm -f gpurun_out/pmc_${TAG}_$name/run_kernel_trace.csv
}
pass mfma SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_mfma gpurun_out/pmc_${TAG}_fetch gpurun_out/pmc_${TAG}_write --top 24 > gpurun_out/pmc_${TAG}_summary.txt 2>&1 || { echo "pmc summary failed"; tail -5 gpurun_out/pmc_${TAG}_summary.txt; exit 1; }
head -30 gpurun_out/pmc_${TAG}_summary.txt
