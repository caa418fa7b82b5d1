"""trilinos_amd -- an MI355X-native (gfx950) Block GMRES hot path with the Belos/Epetra
interface shape.

The product is ``libmigmres.so`` (HIP kernels + host C++ solver behind the C ABI in
``include/migmres.h``); this package is the Python mirror of the reference's
operator/solver interface over that ABI.  Importing it loads the library and fails
loudly if it has not been built -- there is no CPU fallback.
"""

from . import _lib  # noqa: F401  (raises ImportError when libmigmres.so is missing)
from ._lib import MigmresError  # noqa: F401
from .linalg import Comm, CrsMatrix, MultiVector, Operator, galeri_rows, matrix_file_rows, uniform_map  # noqa: F401
from .ifpack2 import Relaxation, Chebyshev  # noqa: F401
from .belos import (BlockGmresSolMgr, PseudoBlockGmresSolMgr, SolverFactory, DGKSOrthoManager, ICGSOrthoManager, LinearProblem, MultiVecTraits,  # noqa: F401
                    OperatorTraits, Converged, Unconverged, TwoNorm, OneNorm, InfNorm, General, Brief)

__all__ = ["MigmresError", "Operator", "Relaxation", "Chebyshev", "galeri_rows", "matrix_file_rows", "PseudoBlockGmresSolMgr", "SolverFactory", "Comm", "CrsMatrix", "MultiVector", "uniform_map", "BlockGmresSolMgr",
           "ICGSOrthoManager", "DGKSOrthoManager", "LinearProblem", "MultiVecTraits", "OperatorTraits",
           "Converged", "Unconverged", "TwoNorm", "OneNorm", "InfNorm", "General", "Brief"]
