"""lssp_amd -- MI355X-native hot path of LSSP (CSR SpMV, fused BLAS-1, ILU
trisolves, BiCGSTAB / GMRES / CG) behind the reference's API.

    from lssp_amd.device import ...   # C-ABI handles (include/lssp_amd.h): Device, DMat, DILU, solve
    from lssp_amd import convert      # CSR / COO / BCSR conversions and transpose on the device
    from lssp_amd.dist import GlooTransport   # host-staged multi-rank transport
    from lssp_amd.synthetic import thermal_like   # config 5's matrix

The reference's own C++ API (lssp_solver_create / _assemble / _solve) reaches
this library through integration/amd_backend.cxx.

The compute lives in lssp_amd/lib/liblssp_amd.so (hand-written HIP for
gfx950).  Importing the package loads it and fails loudly if it is missing.
"""
from . import _lib

_lib.load()

from .device import (BICGSTAB, CG, GMRES, LGMRES, RGMRES, ILUK, ILUT, SERIAL, TREE, DILU, DMat,  # noqa: E402,F401
                     Device, DIdx, DVec, LsspError, comm_unique_id, poisson, solve, sort_columns,
                     BICGSAFE, CGS, GPBICG, CR, CRS, BICRSTAB, BICRSAFE, GPBICR, QMRCGSTAB, TFQMR, ORTHOMIN,
                     BICGSTABL, IDRS)

__all__ = ["Device", "DIdx", "DVec", "DMat", "DILU", "solve", "poisson", "sort_columns", "LsspError",
           "comm_unique_id", "GMRES", "LGMRES", "RGMRES", "BICGSTAB", "CG", "ILUK", "ILUT", "SERIAL", "TREE",
           "BICGSAFE", "CGS", "GPBICG", "CR", "CRS", "BICRSTAB", "BICRSAFE", "GPBICR", "QMRCGSTAB", "TFQMR", "ORTHOMIN",
           "BICGSTABL", "IDRS"]
