// dol_common.h — error plumbing shared by the translation units of libdol_hip.so.
#pragma once

#include <stdint.h>

// The LDS-DMA pipelines (ring_mix_dma / ring_stream_dma / csr_pm / csr_slab /
// the MLP step) retire their loads with counted `s_waitcnt vmcnt(N)` waits
// that also count the buffer stores issued in between, in issue order, and
// the dropped (out-of-range) stores are counted too.  That holds on gfx9
// (one vector-memory counter); targets with a separate store counter (vscnt)
// would make every counted wait wrong.  Device code is built for gfx950 only
// (tests/test_codegen_pins.py pins the emitted waits).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libdol_hip's counted vmcnt pipelines are written for gfx950 (one counter for loads and stores)"
#endif

namespace dol {
// Every size / leading dimension an entry point accepts is at most 2^40
// elements (4 TiB of fp32, far above one GPU's 288 GB), so no byte or block
// count derived from them can overflow int64 (checked under UBSan,
// tests/test_native_abi.py).
constexpr int64_t kMaxDim = int64_t(1) << 40;
extern thread_local char g_err[512];
// Format the thread-local error message and return `code`.
int fail(int code, const char* fmt, ...);
// DOL_OK, or -(hipError_t) of a failed launch (message set).
int check_launch(const char* what);
}  // namespace dol

// First statement of an entry point: reject sizes above kMaxDim.
#define DOL_DIMS_OK(nm, ...)                                                          \
  do {                                                                                \
    for (const int64_t dol_v_ : {__VA_ARGS__})                                        \
      if (dol_v_ > dol::kMaxDim) return dol::fail(DOL_EINVAL, "%s: size above 2^40 elements", nm); \
  } while (0)
