"""simplex_amd — MI355X-native dense simplex pivot engine.

Drop-in for the tableau-pivoting hot path of the-utn-team/simplex-solver
(app/controllers/solver_controller.py:290-363 via simple_simplex).  Kernels are
hand-written HIP for gfx950 in ../csrc, reached through the C-ABI of
include/spx.h (libspx.so, bound by _lib.py).  Submodules:

  engine          DeviceTableau: one tableau resident in HBM, pivot/solve calls
  lp              standard form + two-phase driver
  simple_simplex  create_tableau / add_constraint / add_objective /
                  optimize_json_format (the reference's engine API)
  controller      SolverController with the reference's API surface
  dist            row-sharded tableau across ranks (RCCL over xGMI)
  synth           synthetic LP generators for benchmarks and tests
"""
__version__ = "0.1.0"

from ._lib import SpxLibraryError, lib  # noqa: F401
