"""A caller-owned RCCL communicator from Python (ctypes on the process's librccl.so.1 -- the
copy `import torch` loaded, which librvcp dlopen()s too), for tools that attach one to a
context with rvcp_rccl_attach.  ncclConfig_t follows rccl.h 2.27 (NCCL_CONFIG_INITIALIZER).

  comm = make_comm(world=1, rank=0, blocking=True)   # an ncclComm_t as int
  destroy_comm(comm)
"""
import ctypes
import time

_R = None


class _UID(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


class _Cfg(ctypes.Structure):
    _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                ("blocking", ctypes.c_int), ("cgaClusterSize", ctypes.c_int),
                ("minCTAs", ctypes.c_int), ("maxCTAs", ctypes.c_int), ("netName", ctypes.c_char_p),
                ("splitShare", ctypes.c_int), ("trafficClass", ctypes.c_int),
                ("commName", ctypes.c_char_p), ("collnetEnable", ctypes.c_int),
                ("CTAPolicy", ctypes.c_int), ("shrinkShare", ctypes.c_int),
                ("nvlsCTAs", ctypes.c_int)]


def rccl():
    global _R
    if _R is None:
        import torch  # noqa: F401 -- loads the RCCL librvcp will share
        R = ctypes.CDLL("librccl.so.1")
        R.ncclCommInitRank.argtypes = [ctypes.c_void_p, ctypes.c_int, _UID, ctypes.c_int]
        R.ncclCommInitRankConfig.argtypes = [ctypes.c_void_p, ctypes.c_int, _UID, ctypes.c_int,
                                             ctypes.c_void_p]
        R.ncclCommGetAsyncError.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        R.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        _R = R
    return _R


def make_comm(world=1, rank=0, blocking=True, uid=None):
    """ncclCommInitRank (or ncclCommInitRankConfig with blocking = 0, polled until ready) on the
    current HIP device; returns the ncclComm_t as an int."""
    R = rccl()
    if uid is None:
        uid = _UID()
        if R.ncclGetUniqueId(ctypes.byref(uid)) != 0:
            raise RuntimeError("ncclGetUniqueId failed")
    comm = ctypes.c_void_p()
    if blocking:
        r = R.ncclCommInitRank(ctypes.byref(comm), world, uid, rank)
        if r != 0:
            raise RuntimeError(f"ncclCommInitRank: {r}")
        return comm.value
    ver = ctypes.c_int()
    R.ncclGetVersion(ctypes.byref(ver))
    undef = -2147483648
    cfg = _Cfg(ctypes.sizeof(_Cfg), 0xcafebeef, ver.value, 0, undef, undef, undef, None, undef,
               undef, None, undef, undef, undef, undef)
    r = R.ncclCommInitRankConfig(ctypes.byref(comm), world, uid, rank, ctypes.byref(cfg))
    if r not in (0, 7):
        raise RuntimeError(f"ncclCommInitRankConfig: {r}")
    st, t0 = ctypes.c_int(7), time.perf_counter()
    while st.value == 7 and time.perf_counter() - t0 < 60:
        R.ncclCommGetAsyncError(comm, ctypes.byref(st))
    if st.value != 0:
        raise RuntimeError(f"non-blocking communicator not ready: {st.value}")
    return comm.value


def destroy_comm(comm):
    rccl().ncclCommDestroy(ctypes.c_void_p(comm))
