"""Driven by tests/test_native_abi.py::test_argument_validation_under_asan_ubsan in a
subprocess with the ASan runtime preloaded: loads the host-sanitised
libdol_hip_asan.so and calls every C-ABI entry point with arguments its
validation must reject (NULL pointers, negative sizes, sizes whose byte counts
overflow, misaligned or aliased buffers).  Nothing here reaches a kernel
launch; ASan / UBSan abort the process on any host-side memory error or
undefined behaviour (signed overflow, bad shifts) on these paths."""
import ctypes
import sys

sys.path[:0] = sys.argv[2:]
from dolhip import _native  # noqa: E402

L = ctypes.CDLL(sys.argv[1])
for name, argtypes in _native.SIGNATURES.items():
    fn = getattr(L, name)
    fn.argtypes = argtypes
    fn.restype = _native._RESTYPES.get(name, ctypes.c_int)

FAKE = 1 << 20  # a 16-B aligned address that is never dereferenced


def vals(argtypes, mode):
    out = []
    for k, t in enumerate(argtypes):
        if t is ctypes.c_void_p:
            out.append(None if mode == "null" else FAKE + 4096 * k)
        elif t is ctypes.c_float:
            out.append(0.1)
        elif t is ctypes.c_uint64:
            out.append(7)
        elif t is ctypes.c_int64:
            out.append({"null": 8, "neg": -3, "huge": (1 << 62) + 4, "odd": 7}[mode])
        else:  # int32 / int
            out.append({"null": 8, "neg": -3, "huge": (1 << 31) - 1, "odd": 7}[mode])
    return out


calls = 0
for name, argtypes in _native.SIGNATURES.items():
    if name in ("dol_version", "dol_last_error", "dol_csr_slab_nk"):  # queries without failure modes
        continue
    for mode in ("null", "neg", "huge", "odd"):
        rc = getattr(L, name)(*vals(argtypes, mode))
        calls += 1
        if _native._RESTYPES.get(name) is ctypes.c_int64:
            continue  # workspace-size queries: only must not trip a sanitizer
        if name == "dol_pm_set_stage_order":  # a setter: 8 / 7 are valid settings, -3 / 2^31-1 are not
            if (mode in ("neg", "huge")) != (rc == -1):
                print(f"{name}: {mode} gave rc={rc}")
                sys.exit(5)
            L.dol_pm_set_stage_order(0)
            continue
        if name == "dol_bank_free" and mode == "null":  # free(NULL) is a no-op, like free()
            if rc != 0:
                print(f"{name}(NULL) gave rc={rc}")
                sys.exit(6)
            continue
        if mode in ("null", "neg") and rc != -1:
            print(f"{name} accepted {mode} arguments (rc={rc})")
            sys.exit(3)
        if rc == 0 and mode == "huge":
            print(f"{name} accepted huge sizes")
            sys.exit(4)
print(f"asan-abi ok: {calls} rejected calls")
