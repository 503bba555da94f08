"""nts — MI355X-native sampled-GNN hot path (drop-in for the reference's
FastSampler / ntsGraphOp / NtsContext surface).

Layout:
  _abi.py       ctypes binding of the C-ABI (include/nts_hip.h, libnts_hip.so)
  hip.py        thin Python handle over the C-ABI (kernel-level tests, data prep)
  host/         C++ (libtorch) host layer mirroring the reference classes
  dataloader.py reference on-disk formats + cfg parser
  synthetic.py  BASELINE-shaped synthetic graphs
"""
import torch  # noqa: F401  load torch's HIP runtime before libnts_hip.so

__all__ = ["_abi", "hip", "dataloader", "synthetic"]
