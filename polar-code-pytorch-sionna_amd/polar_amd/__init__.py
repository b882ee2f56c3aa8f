"""polar_amd -- MI355X-native (gfx950) SC / SC-list polar decoding behind the reference API.

Hot path: libpolar_mi355x.so (hand-written HIP kernels + C ABI, include/polar_mi355x.h).
Drop-ins: SC_Dec / SCL_Dec (x_run_sn_polar/polar/polar_sc.py, polar_scl.py); the my_sn API in
polar_amd.mysn (decoders), polar_amd.polar5g (encoders, 5G wrapper, frozen-set helpers) and
polar_amd.crc (CRCEncoder / CRCDecoder / int_mod_2).
"""
from . import _lib, ops  # noqa: F401
from .decoders import SC_Dec, SCL_Dec  # noqa: F401
from .crc import CRCDecoder, CRCEncoder, int_mod_2  # noqa: F401
from .frozen import F2, get_Kern_frozen_bits, reference_frozen_pos, frozen_mask  # noqa: F401

__all__ = ["SC_Dec", "SCL_Dec", "F2", "get_Kern_frozen_bits", "reference_frozen_pos", "frozen_mask", "ops",
           "CRCEncoder", "CRCDecoder", "int_mod_2"]
