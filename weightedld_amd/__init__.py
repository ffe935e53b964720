"""weightedld_amd — MI355X-native WeightedLD all-pairs LD hot path.

Python mirror of the weighted_ld crate surface (rust/weighted_ld/src/lib.rs)
over the C ABI in include/weightedld.h.  The hot path
(all_weighted_ld_pairs / single_weighted_ld_pair) runs only on a gfx950 GPU;
there is no CPU fallback.
"""
from ._lib import LIB_PATH, WldError, lib  # noqa: F401
from .api import *  # noqa: F401,F403
from .api import __all__ as _api_all

__all__ = list(_api_all) + ["LIB_PATH", "lib"]
__version__ = "0.1.0"
