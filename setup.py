"""Build the in-tree native extensions for MI355X (gfx950).

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

* ``dalle_amd._C``       -- hand-written HIP/CDNA4 kernels (csrc/kernels, csrc/optim) + torch bindings
* ``dalle_amd._kvstore`` -- C++ TCP key-value store with subkeys / expiration (the DHT replacement)
* ``dalle_amd._tokenizer`` -- C++ SentencePiece-unigram caption tokenizer (the Rust ``tokenizers`` replacement)
"""
import os

from setuptools import Extension, setup
from torch.utils.cpp_extension import BuildExtension, CppExtension, include_paths, library_paths

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
ROOT = os.path.dirname(os.path.abspath(__file__))

hip_sources = [
    "csrc/binding.cpp",
    "csrc/kernels/attention.hip",
    "csrc/kernels/attention_fused.hip",
    "csrc/kernels/rotary.hip",
    "csrc/kernels/layernorm_shift.hip",
    "csrc/kernels/elementwise.hip",
    "csrc/kernels/xent.hip",
    "csrc/kernels/decode.hip",
    "csrc/kernels/gemm.hip",
    "csrc/kernels/gemm_pt.hip",
    "csrc/kernels/quant.hip",
    "csrc/kernels/skinny.hip",
    "csrc/kernels/sample.hip",
    "csrc/kernels/powersgd.hip",
    "csrc/kernels/embed.hip",
    "csrc/kernels/conv.hip",
    "csrc/optim/lamb.hip",
    "csrc/asm/asm_gemm.cpp",
]

# the hand-scheduled assembly kernels: generate + assemble + embed (csrc/asm/gemm_hsaco.inc) before compiling
import subprocess, sys  # noqa: E401,E402

subprocess.run([sys.executable, os.path.join(ROOT, "csrc/asm/build_asm.py")], check=True)

# Plain setuptools Extension (not CUDAExtension): CUDAExtension would run hipify over the sources.
# These kernels are written for CDNA4 directly; BuildExtension compiles the .hip files with hipcc.
ext_modules = [
    Extension(
        "dalle_amd._C",
        hip_sources,
        include_dirs=[os.path.join(ROOT, "csrc")] + include_paths(device_type="cuda"),
        library_dirs=library_paths(device_type="cuda"),
        libraries=["c10", "torch", "torch_cpu", "torch_python", "amdhip64", "c10_hip", "torch_hip", "hipblaslt"],
        language="c++",
        extra_compile_args={
            "cxx": ["-O3", "-std=c++17", "-g0"],
            "nvcc": ["-O3", "--offload-arch=gfx950", "-std=c++17", "-munsafe-fp-atomics", "-g0"],
        },
        extra_link_args=["-s"],   # no host debug info: 21 MB -> the ~4 MB of code and embedded code objects
    ),
]

if os.path.exists(os.path.join(ROOT, "csrc/store/kvstore.cpp")):
    ext_modules.append(
        CppExtension(
            "dalle_amd._kvstore",
            ["csrc/store/kvstore.cpp"],
            extra_compile_args=["-O2", "-std=c++17", "-g0"],
            extra_link_args=["-s"],
        )
    )

# plain pybind11 module: no torch / HIP libraries, so the data-loader can import it on its own
import pybind11  # noqa: E402

ext_modules.append(
    Extension(
        "dalle_amd._tokenizer",
        ["csrc/tokenizer/tokenizer.cpp"],
        include_dirs=[os.path.join(ROOT, "csrc/tokenizer"), pybind11.get_include()],
        language="c++",
        extra_compile_args={"cxx": ["-O2", "-std=c++17", "-fvisibility=hidden", "-g0"]},
        extra_link_args=["-pthread", "-s"],
    )
)

setup(
    name="dalle_amd",
    version="0.1.0",
    packages=["dalle_amd"],
    ext_modules=ext_modules,
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
