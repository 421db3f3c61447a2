# same-box A/B of two builds of the extension: the tree's dalle_amd/_C*.so ("new") against ab/_C_old.so ("old"),
# run from a copy of the tree with the old library swapped in. usage: bash scripts/gpu_ab_so.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=/tmp/ab_old_tree
rm -rf $OLD && mkdir -p $OLD && cp -r bench.py benchmarks dalle_amd csrc $OLD/ && cp ab/_C_old.so $OLD/dalle_amd/_C.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for v in new old new old; do
  d=$PWD; [ $v = old ] && d=$OLD
  (cd $d && timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128) > gpurun_out/ab_parts_$v.log 2>&1 || { echo "parts $v failed"; tail -5 gpurun_out/ab_parts_$v.log; exit 1; }
  echo "$v $(grep -h 'bench24_attention' gpurun_out/ab_parts_$v.log) $(grep -h axial_row gpurun_out/ab_parts_$v.log)"
done
for v in new old new old; do
  d=$PWD; [ $v = old ] && d=$OLD
  (cd $d && timeout -k 10 300 python3 bench.py --steps 10 --warmup 3) > gpurun_out/ab_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab_bench_$v.log; exit 1; }
  echo "bench $v $(grep '^{' gpurun_out/ab_bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
