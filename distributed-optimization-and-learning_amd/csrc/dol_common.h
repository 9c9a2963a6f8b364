// dol_common.h — error plumbing shared by the translation units of libdol_hip.so.
#pragma once

namespace dol {
extern thread_local char g_err[512];
// Format the thread-local error message and return `code`.
int fail(int code, const char* fmt, ...);
// DOL_OK, or -(hipError_t) of a failed launch (message set).
int check_launch(const char* what);
}  // namespace dol
