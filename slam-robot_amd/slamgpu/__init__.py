"""slamgpu — Python bindings for the MI355X-native local-mapping back end (libslamgpu.so).

The compute lives in HIP kernels behind the C-ABI in include/slamgpu.h; this package only marshals
numpy arrays across it (ctypes) and generates seeded synthetic scenes for tests and benchmarks.
"""
from .capi import (ProblemArrays, SgDeviceOptions, SgMap, SgProblem, SgSolverOptions,  # noqa: F401
                   SgSolverSummary, SlamGpuError, default_solver_options, load_library)
from .scene import CONFIGS, MapArrays, make_config, make_scene  # noqa: F401
