// Error plumbing and small C-ABI queries of libgsamd.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/gsamd.h"

namespace gs {

static thread_local char t_err[1024] = "";

void set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t_err, sizeof(t_err), fmt, ap);
    va_end(ap);
}

int hip_fail(hipError_t e, const char *what, const char *file, int line)
{
    set_error("%s: %s (%s:%d)", what, hipGetErrorString(e), file, line);
    return GS_E_HIP;
}

}  // namespace gs

extern "C" int gs_abi_version(void) { return GS_ABI_VERSION; }

extern "C" const char *gs_last_error(void) { return gs::t_err; }

// the kernel sources' hashes, computed by build_lib.py (gsamd/buildinfo.source_hash) when this file
// is compiled; build_lib.py recompiles it whenever a hash changes
#ifndef GS_SRC_HASH_MLP
#define GS_SRC_HASH_MLP "unknown"
#endif
#ifndef GS_SRC_HASH_CNN
#define GS_SRC_HASH_CNN "unknown"
#endif
#ifndef GS_SRC_HASH_ALL
#define GS_SRC_HASH_ALL "unknown"
#endif

extern "C" const char *gs_build_source_hash(const char *path)
{
    if (!path || !*path) return GS_SRC_HASH_ALL;
    if (!strcmp(path, "mlp")) return GS_SRC_HASH_MLP;
    if (!strcmp(path, "cnn")) return GS_SRC_HASH_CNN;
    return nullptr;
}
