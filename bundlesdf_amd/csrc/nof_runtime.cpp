// Host runtime pieces of libnof: error reporting, level tables, version.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "nof_device.h"

namespace nof {

static thread_local char g_err[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(NOF_ELAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
    return NOF_OK;
}

// gridencoder.cu:155-156 — `exp2f(level * S) * H - 1.0f` (contracted to an
// FMA by nvcc's default --fmad=true), resolution = ceil(scale) + 1.
void level_params(uint32_t L, float S, uint32_t H, LevelParams &lp) {
    for (uint32_t l = 0; l < L && l < NOF_MAX_LEVELS; ++l) {
        float sc = fmaf(exp2f((float)l * S), (float)H, -1.0f);
        lp.scale[l] = sc;
        lp.res[l] = (uint32_t)ceilf(sc) + 1u;
    }
}

}  // namespace nof

extern "C" {

const char *nof_last_error(void) { return nof::g_err; }

const char *nof_version(void) { return "nof 0.1 gfx950 (hipcc " __clang_version__ ")"; }

void nof_level_params(uint32_t L, float S, uint32_t H, float *scales, uint32_t *resolutions) {
    nof::LevelParams lp;
    nof::level_params(L, S, H, lp);
    for (uint32_t l = 0; l < L && l < NOF_MAX_LEVELS; ++l) {
        scales[l] = lp.scale[l];
        resolutions[l] = lp.res[l];
    }
}

void nof_level_table(uint32_t L, float S, uint32_t H, const int32_t *offsets_host, float *table_host) {
    nof::LevelParams lp;
    nof::level_params(L, S, H, lp);
    for (uint32_t l = 0; l < L && l < NOF_MAX_LEVELS; ++l) {
        uint32_t res = lp.res[l], off = (uint32_t)offsets_host[l], rows = (uint32_t)(offsets_host[l + 1] - offsets_host[l]);
        table_host[l * 4 + 0] = lp.scale[l];
        memcpy(&table_host[l * 4 + 1], &res, 4);
        memcpy(&table_host[l * 4 + 2], &off, 4);
        memcpy(&table_host[l * 4 + 3], &rows, 4);
    }
}

}  // extern "C"
