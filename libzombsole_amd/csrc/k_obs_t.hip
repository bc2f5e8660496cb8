// k_obs_t.hip — every observation kernel (zs_obs.hpp) for one output dtype, compiled once per dtype
// (-DZS_OBS_T=0 int32, 1 int64, 2 int16).
#include "zs_launch.hpp"
#include "zs_obs.hpp"

#ifndef ZS_OBS_T
#error "compile with -DZS_OBS_T=<ZS_DTYPE_*>"
#endif
#if ZS_OBS_T == 1
typedef int64_t TT;
#define ZS_OBS_FN(f) f##_i64
#elif ZS_OBS_T == 0
typedef int32_t TT;
#define ZS_OBS_FN(f) f##_i32
#else
typedef int16_t TT;
#define ZS_OBS_FN(f) f##_i16
#endif

template <int NB>
static void launch_nb(const ObsLaunch& o, hipStream_t s, const Dev& d) {
    TT* out = (TT*)o.obs;
    const dim3 g(o.grid), b(o.block);
    switch (o.kind) {
    case OBSK_RING:
        if (o.patched) hipLaunchKernelGGL((k_obs_ring<TT, NB, true>), g, b, o.lds, s, d, out, o.L, o.env0, o.env1);
        else hipLaunchKernelGGL((k_obs_ring<TT, NB, false>), g, b, o.lds, s, d, out, o.L, o.env0, o.env1);
        break;
    case OBSK_BRING: hipLaunchKernelGGL((k_obs_pbring<TT, NB>), g, b, o.lds, s, d, out, o.env0, o.env1, o.us); break;
    case OBSK_PATCH: hipLaunchKernelGGL((k_obs_patch<TT, NB>), g, b, o.lds, s, d, out, o.env0, o.env1); break;
    case OBSK_PIPE: hipLaunchKernelGGL((k_obs_pipe<TT, NB>), g, b, o.lds, s, d, out, o.L, o.env0, o.env1); break;
    default: hipLaunchKernelGGL((k_obs_gather<TT, NB>), g, b, o.lds, s, d, out, o.mask, o.L, o.stat); break;
    }
}

hipError_t ZS_OBS_FN(launch_obs)(const ObsLaunch& o, hipStream_t s, const Dev& d) {
    if (o.kind == OBSK_OBS)
        hipLaunchKernelGGL(k_obs<TT>, dim3(o.grid), dim3(o.block), o.lds, s, d, (TT*)o.obs, o.mask, o.L, o.stat);
    else if (o.nobs == 1) launch_nb<1>(o, s, d);
    else if (o.nobs == 2) launch_nb<2>(o, s, d);
    else if (o.nobs == 4) launch_nb<4>(o, s, d);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

// raise a kernel's dynamic-LDS limit past 64 KiB (k_obs_ring / k_obs_patch / k_obs_pbring)
hipError_t ZS_OBS_FN(obs_lds_attr)(int kind, int nobs, int patched, int bytes) {
    const void* fn = nullptr;
#define ZS_FN3(K) (nobs == 1 ? (const void*)K<TT, 1> : nobs == 2 ? (const void*)K<TT, 2> : (const void*)K<TT, 4>)
    if (kind == OBSK_PATCH) {
        fn = ZS_FN3(k_obs_patch);
    } else if (kind == OBSK_BRING) {
        fn = ZS_FN3(k_obs_pbring);
    } else if (kind == OBSK_RING) {
        if (patched)
            fn = nobs == 1 ? (const void*)k_obs_ring<TT, 1, true>
                 : nobs == 2 ? (const void*)k_obs_ring<TT, 2, true> : (const void*)k_obs_ring<TT, 4, true>;
        else
            fn = nobs == 1 ? (const void*)k_obs_ring<TT, 1, false>
                 : nobs == 2 ? (const void*)k_obs_ring<TT, 2, false> : (const void*)k_obs_ring<TT, 4, false>;
    } else {
        return hipErrorInvalidValue;
    }
#undef ZS_FN3
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
