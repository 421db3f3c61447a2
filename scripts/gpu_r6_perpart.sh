# round 6: per-part linear decode graphs (default) vs the joint two-branch graph: generation tests, host-submit probe,
# and bench_inference A/B (distinct captions and run_inference's repeated caption), alternating on one box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py tests/test_serve_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6pp_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r6pp_pytest.log | head -30; tail -30 gpurun_out/r6pp_pytest.log; exit 1; }
tail -1 gpurun_out/r6pp_pytest.log
for mode in per-part joint; do
  DALLE_AMD_DECODE_GRAPHS=$mode timeout -k 10 240 python3 benchmarks/probe_replay_host.py > gpurun_out/r6pp_probe_$mode.log 2>&1 || { echo "probe $mode failed"; tail -5 gpurun_out/r6pp_probe_$mode.log; exit 1; }
  echo "probe $mode $(grep '^{' gpurun_out/r6pp_probe_$mode.log)"
done
for rep in 1 2; do
  for mode in per-part joint; do
    for cap in "" "--same-caption"; do
      DALLE_AMD_DECODE_GRAPHS=$mode timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --iters 4 $cap > gpurun_out/r6pp_gen.log 2>&1 || { echo "gen $mode $cap failed"; tail -5 gpurun_out/r6pp_gen.log; exit 1; }
      echo "gen mode=$mode cap=${cap:-distinct} $(grep -E '^# generate' gpurun_out/r6pp_gen.log | tr '\n' ' ') $(grep '^{' gpurun_out/r6pp_gen.log | grep -oE '"value": [0-9.]+|"seconds_per_batch": [0-9.]+|"ms_per_decode_step": [0-9.]+|"sampling_seconds": [0-9.]+' | tr '\n' ' ')"
    done
  done
done
