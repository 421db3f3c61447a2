set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -m pytest tests -m gpu -q > gpurun_out/pytest_gpu_full.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
printf 'a red apple on a table\nthe northern lights over a snowy forest\n' > /tmp/queries.txt
timeout -k 10 600 python3 inference/run_inference.py --queries /tmp/queries.txt --output-dir gpurun_out/inf_out --model-preset reference --batch-size 16 --n-iters 1 --top-k 256 --clip random > gpurun_out/run_inference.log 2>&1 || { echo "run_inference failed"; tail -20 gpurun_out/run_inference.log; exit 1; }
tail -5 gpurun_out/run_inference.log
ls -la gpurun_out/inf_out
