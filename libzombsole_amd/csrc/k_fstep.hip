// k_fstep.hip — the one-launch step (zs_fstep.hpp) for the shapes it is instantiated for:
// lanes per env G, observation dtype and observations per env (C3: 8 / int64 / 2, C5: 16 / int16 / 4).
#include "zs_fstep.hpp"

template <int G, typename T, int NOBS>
static hipError_t fs_go(unsigned grid, hipStream_t s, const Dev& d, const FsArgs& a) {
    hipLaunchKernelGGL((k_fstep<G, T, NOBS>), dim3(grid), dim3(64 * FS_WAVES), a.L.bytes, s, d, a);
    return hipGetLastError();
}

template <int G, typename T, int NOBS>
static hipError_t fs_attr(int bytes) {
    return hipFuncSetAttribute((const void*)k_fstep<G, T, NOBS>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

#define FS_SHAPES(X)              \
    X(8, ZS_DTYPE_I64, int64_t, 2) \
    X(16, ZS_DTYPE_I64, int64_t, 2) \
    X(16, ZS_DTYPE_I16, int16_t, 4)

hipError_t launch_fstep(int G, int dtype, int nobs, unsigned grid, hipStream_t s, const Dev& d, const FsArgs& a) {
#define FS_LAUNCH(g, dt, t, n) \
    if (G == g && dtype == dt && nobs == n) return fs_go<g, t, n>(grid, s, d, a);
    FS_SHAPES(FS_LAUNCH)
#undef FS_LAUNCH
    return hipErrorNotSupported;
}

hipError_t fstep_attr(int G, int dtype, int nobs, int bytes) {
#define FS_ATTR(g, dt, t, n) \
    if (G == g && dtype == dt && nobs == n) return fs_attr<g, t, n>(bytes);
    FS_SHAPES(FS_ATTR)
#undef FS_ATTR
    return hipErrorNotSupported;
}
