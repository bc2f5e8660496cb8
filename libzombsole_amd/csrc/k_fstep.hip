// k_fstep.hip — the one-launch step (zs_fstep.hpp) for the shapes it is instantiated for: lanes per env G,
// observation dtype, observations per env, and the role shape (tick, encoder, writer waves per workgroup).
#include "zs_fstep.hpp"

// one-round shapes (eight tick waves, one unit each) load the tick's RNG window early
template <int G, typename T, int NOBS, int NT, int NEN, int NW>
static hipError_t fs_go(unsigned grid, hipStream_t s, const Dev& d, const FsArgs& a) {
    hipLaunchKernelGGL((k_fstep<G, T, NOBS, NT, NEN, NW, (NT >= 8)>), dim3(grid), dim3(64 * (NT + NEN + NW)), a.L.bytes, s,
                       d, a);
    return hipGetLastError();
}

template <int G, typename T, int NOBS, int NT, int NEN, int NW>
static hipError_t fs_attr(int bytes) {
    return hipFuncSetAttribute((const void*)k_fstep<G, T, NOBS, NT, NEN, NW, (NT >= 8)>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// (G, dtype, T, observations per env, tick / encoder / writer waves)
#ifndef FS_SHAPES
#define FS_SHAPES(X)                         \
    X(8, ZS_DTYPE_I64, int64_t, 2, 4, 9, 3)  \
    X(8, ZS_DTYPE_I64, int64_t, 2, 6, 7, 3)  \
    X(16, ZS_DTYPE_I16, int16_t, 4, 4, 9, 3) \
    X(16, ZS_DTYPE_I16, int16_t, 4, 6, 7, 3) \
    X(16, ZS_DTYPE_I64, int64_t, 2, 8, 5, 3) \
    X(16, ZS_DTYPE_I64, int64_t, 2, 8, 6, 2) \
    X(16, ZS_DTYPE_I16, int16_t, 4, 8, 5, 3)
#endif

hipError_t launch_fstep(int G, int dtype, int nobs, FsShape sh, unsigned grid, hipStream_t s, const Dev& d,
                        const FsArgs& a) {
#define FS_LAUNCH(g, dt, t, n, vt, ve, vw)                                                 \
    if (G == g && dtype == dt && nobs == n && sh.nt == vt && sh.nen == ve && sh.nw == vw) \
        return fs_go<g, t, n, vt, ve, vw>(grid, s, d, a);
    FS_SHAPES(FS_LAUNCH)
#undef FS_LAUNCH
    return hipErrorNotSupported;
}

hipError_t fstep_attr(int G, int dtype, int nobs, FsShape sh, int bytes) {
#define FS_ATTR(g, dt, t, n, vt, ve, vw)                                                   \
    if (G == g && dtype == dt && nobs == n && sh.nt == vt && sh.nen == ve && sh.nw == vw) \
        return fs_attr<g, t, n, vt, ve, vw>(bytes);
    FS_SHAPES(FS_ATTR)
#undef FS_ATTR
    return hipErrorNotSupported;
}
