"""dspcore — MI355X-native hot path of Renatovela-ctrl/dsp-audio-project.

Layers (bottom-up):
  libdspcore.so   hand-written gfx950 HIP kernels behind a C-ABI (include/dspcore.h)
  _lib            ctypes binding of that ABI
  design          host-side float64 filter design / call planning (reference rules)
  ops             per-kernel device operators on torch CUDA tensors
  chain           batched SRC -> EQ -> spectrum plan (the benchmarked path)
  shard           one host thread per GPU over contiguous channel ranges
  host            numpy batches through the chain with PCIe copies overlapped
The reference-compatible drop-in is dsp-audio-project_amd/modules/dsp_core.py.
"""
from . import design  # noqa: F401

__all__ = ["design", "ops", "chain", "shard", "host"]
__version__ = "1.6.0"


def __getattr__(name):  # lazy: importing design must not require the GPU library
    if name in ("ops", "chain", "shard", "host", "_lib"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
