"""dmclock_amd -- MI355X-native dmClock server queue.

The product is the HIP engine behind the C-ABI of include/dmclock_gpu.h
(dmclock_amd/libdmclock_gpu.so) and the C++ facade
dmclock_amd/include/dmclock_server.h that re-exports the reference's
crimson::dmclock API on top of it.  This Python package is the ctypes binding
used by the tests and by bench.py.
"""
from ._abi import (AT_LIMIT_ALLOW, AT_LIMIT_REJECT, AT_LIMIT_WAIT,  # noqa: F401
                   DECISION_DTYPE, NEXT_FUTURE, NEXT_NONE, NEXT_RETURNING,
                   PHASE_PRIORITY, PHASE_RESERVATION, REQUEST_DTYPE,
                   make_requests)

__all__ = ["GpuQueue", "REQUEST_DTYPE", "DECISION_DTYPE", "make_requests"]


def __getattr__(name):
    if name == "GpuQueue":
        from .gpu import GpuQueue
        return GpuQueue
    raise AttributeError(name)
