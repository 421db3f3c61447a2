set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_kernels_gpu.py -q -x -k "uniform8bit" > gpurun_out/pytest_quant.log 2>&1 || { echo "pytest quant failed"; tail -40 gpurun_out/pytest_quant.log; exit 1; }
tail -2 gpurun_out/pytest_quant.log
timeout -k 10 300 python3 -c "
import torch, time
from dalle_amd.parallel.compression import Uniform8BitQuantization
x = torch.randn(125_000_000, device='cuda')
c = Uniform8BitQuantization()
for _ in range(2): c.compress(x)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(5): r = c.compress(x)
torch.cuda.synchronize(); print('uq8 compress 125M elems: %.3f ms' % ((time.perf_counter() - t) / 5 * 1e3))
" > gpurun_out/quant_bench.log 2>&1 || { echo "quant bench failed"; tail -5 gpurun_out/quant_bench.log; exit 1; }
grep compress gpurun_out/quant_bench.log
