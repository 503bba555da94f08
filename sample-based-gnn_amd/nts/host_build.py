"""Build the C++ host layer (libtorch-ROCm + pybind11) in-tree.

The extension links libnts_hip.so (the C-ABI) and torch's own HIP runtime;
it is written to nts/lib/ so it travels with the repository snapshot.
"""
from __future__ import annotations

import os
import pathlib

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]
SRC = HERE / "host"
LIB = HERE / "lib"
BUILD = LIB / "host_build"
NAME = "nts_host_ext"


def build(verbose: bool = False):
    import torch
    from torch.utils import cpp_extension

    BUILD.mkdir(parents=True, exist_ok=True)
    torch_lib = pathlib.Path(torch.__file__).parent / "lib"
    os.environ.setdefault("MAX_JOBS", str(min(os.cpu_count() or 8, 16)))
    mod = cpp_extension.load(
        name=NAME,
        sources=[str(SRC / f) for f in ("core.cpp", "gcn.cpp", "bindings.cpp")],
        extra_include_paths=[str(ROOT / "include"), str(SRC), "/opt/rocm/include"],
        extra_cflags=["-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                      "-Wno-unused-variable"],
        extra_ldflags=[f"-L{LIB}", "-lnts_hip", f"-L{torch_lib}", "-lc10_hip",
                       "-Wl,-rpath,$ORIGIN/..", f"-Wl,-rpath,{LIB}"],
        build_directory=str(BUILD),
        with_cuda=False,
        verbose=verbose,
    )
    return mod
