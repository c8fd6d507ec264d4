// Error plumbing and small C-ABI queries of libgsamd.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

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
