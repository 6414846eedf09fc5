"""What the HIP runtime and ROCr still know about a host address range.

Test helper for the registration lifecycle (Weak #1): after
rs_host_register -> rs_host_unregister, no page of the range may still be
registered with either runtime layer, or a later pageable copy from a new
allocation at those addresses could be served through a stale mapping.

  * hipPointerGetAttributes: the HIP runtime's memory-object map
    (hipMemoryTypeHost = registered or pinned host memory);
  * hsa_amd_pointer_info: ROCr's view (HSA_EXT_POINTER_TYPE_LOCKED = a range
    locked through ROCr; HSA = a runtime allocation).

Calibrated on the MI355X box (tools/ptr_state_probe.py,
profiles/r06/ptr_state_probe.log): a hipHostRegister'ed page (directly or
through rs_host_register) is hipMemoryTypeHost to HIP and UNKNOWN to ROCr
(the runtime registers user memory below ROCr's allocation map), a pageable
page is hipMemoryTypeUnregistered / UNKNOWN, a hipHostMalloc'ed one is Host /
HSA.  So "registered" is HIP's answer; ROCr's LOCKED is still reported where
it appears.  Both are host-side queries: no GPU work is enqueued.
"""
import ctypes
import mmap

PAGE = mmap.PAGESIZE
HSA_LOCKED = 2
HIP_HOST = 1


class _PtrInfo(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint32), ("type", ctypes.c_uint32), ("agentBaseAddress", ctypes.c_void_p),
                ("hostBaseAddress", ctypes.c_void_p), ("sizeInBytes", ctypes.c_size_t),
                ("userData", ctypes.c_void_p), ("agentOwner", ctypes.c_uint64), ("global_flags", ctypes.c_uint32),
                ("registered", ctypes.c_bool)]


class _HipAttr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


_LIBS = []


def _libs():
    if not _LIBS:
        hip = ctypes.CDLL("libamdhip64.so")
        hsa = ctypes.CDLL("libhsa-runtime64.so.1")
        hip.hipPointerGetAttributes.argtypes = [ctypes.POINTER(_HipAttr), ctypes.c_void_p]
        hip.hipGetLastError.restype = ctypes.c_int
        hsa.hsa_amd_pointer_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(_PtrInfo), ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]
        _LIBS.extend([hip, hsa])
    return _LIBS


def page_state(addr: int):
    """(rocr type, rocr base, rocr size, hip type) of the page holding addr;
    a negative type is the call's error code."""
    hip, hsa = _libs()
    pi = _PtrInfo()
    pi.size = ctypes.sizeof(_PtrInfo)
    rc = hsa.hsa_amd_pointer_info(ctypes.c_void_p(addr), ctypes.byref(pi), None, None, None)
    rt = pi.type if rc == 0 else -rc
    ha = _HipAttr()
    hrc = hip.hipPointerGetAttributes(ctypes.byref(ha), ctypes.c_void_p(addr))
    if hrc != 0:
        hip.hipGetLastError()
    return rt, (pi.hostBaseAddress or 0) if rt > 0 else 0, pi.sizeInBytes if rt > 0 else 0, (
        ha.type if hrc == 0 else -hrc)


def known_pages(lo: int, hi: int, skip=()):
    """Pages of [lo, hi) that either layer still reports as registered / pinned
    host memory (pages whose start is in `skip` are not asked)."""
    out = []
    for pg in range(lo & ~(PAGE - 1), hi, PAGE):
        if pg in skip:
            continue
        rt, base, size, ht = page_state(pg)
        if rt == HSA_LOCKED or ht == HIP_HOST:
            out.append((hex(pg), rt, hex(base), size, ht))
    return out


def registered(addr: int) -> bool:
    return page_state(addr)[3] == HIP_HOST


_GPUS = []


def _gpu_agents():
    if not _GPUS:
        hsa = _libs()[1]
        cb_t = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)

        def on_agent(agent, _data):
            kind = ctypes.c_uint32(0)
            hsa.hsa_agent_get_info(ctypes.c_uint64(agent), 17, ctypes.byref(kind))  # HSA_AGENT_INFO_DEVICE
            if kind.value == 1:  # HSA_DEVICE_TYPE_GPU
                _GPUS.append(agent)
            return 0

        cb = cb_t(on_agent)
        hsa.hsa_iterate_agents(cb, None)
    return _GPUS


class _SvmPair(ctypes.Structure):
    _fields_ = [("attribute", ctypes.c_uint64), ("value", ctypes.c_uint64)]


def gpu_access(addr: int) -> str:
    """KFD's shared-virtual-memory view of the page holding addr for the first
    GPU (hsa_amd_svm_attributes_get, HSA_AMD_SVM_ATTRIB_ACCESS_QUERY):
    "in-place" (GPU-mapped, what hipHostRegister sets), "accessible",
    "no-access" (a never-registered page) or "unknown" (no SVM API / error)."""
    hsa = _libs()[1]
    gpus = _gpu_agents()
    if not gpus:
        return "unknown"
    hsa.hsa_amd_svm_attributes_get.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_SvmPair),
                                               ctypes.c_size_t]
    pr = (_SvmPair * 1)((0x203, gpus[0]))
    if hsa.hsa_amd_svm_attributes_get(ctypes.c_void_p(addr & ~(PAGE - 1)), PAGE, pr, 1) != 0:
        return "unknown"
    return {0x200: "accessible", 0x201: "in-place", 0x202: "no-access"}.get(pr[0].attribute, "unknown")


def gpu_mapped_pages(lo: int, hi: int):
    """Whole pages inside [lo, hi) that KFD still maps for the GPU in place."""
    first = (lo + PAGE - 1) & ~(PAGE - 1)
    return [hex(pg) for pg in range(first, hi - PAGE + 1, PAGE) if gpu_access(pg) == "in-place"]



def gpu_revoke(lo: int, hi: int) -> bool:
    """Set KFD's SVM access of the whole pages inside [lo, hi) to no-access
    for every GPU (hsa_amd_svm_attributes_set, what rs_host_unregister's
    revoke does), so a test can start from pages no earlier copy left
    GPU-mapped.  False when the SVM API is missing or refuses."""
    hsa = _libs()[1]
    gpus = _gpu_agents()
    first, last = (lo + PAGE - 1) & ~(PAGE - 1), hi & ~(PAGE - 1)
    if not gpus or last <= first:
        return False
    hsa.hsa_amd_svm_attributes_set.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_SvmPair),
                                               ctypes.c_size_t]
    prs = (_SvmPair * len(gpus))(*[(0x202, g) for g in gpus])
    return hsa.hsa_amd_svm_attributes_set(ctypes.c_void_p(first), last - first, prs, len(gpus)) == 0
