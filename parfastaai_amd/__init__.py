"""parfastaai_amd -- MI355X-native all-pairs AJI engine (drop-in for ParFastAAI's hot path).

Host-side mirror of the reference's interfaces over the C ABI of
libpfaai_hip.so (include/pfaai_hip.h):
  datastruct  DataStructInterface modes (ds_impl.hpp)      -- arrays + index maps
  impl        ParFAAIImpl (algorithm_impl.hpp)              -- run/getJAC/getAJI on the GPU
  loader      SQLite SCP/tetramer loader (scp_db.hpp, db_helper.hpp)
  formats     cereal fixtures / outputs, CSV matrix (main.cpp:133-175)
  syn         synthetic SCP/tetramer databases
"""
from . import _capi  # noqa: F401  (imports torch first when present: one HIP runtime)
from .datastruct import ParFAAIData, ParFAAIQSubData, ParFAAIQryTgtData  # noqa: F401
from .impl import ParFAAIImpl  # noqa: F401

__all__ = ["ParFAAIData", "ParFAAIQSubData", "ParFAAIQryTgtData", "ParFAAIImpl"]
