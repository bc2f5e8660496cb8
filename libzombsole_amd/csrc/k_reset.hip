// k_reset.hip — the reset-work kernels (zs_reset.hpp): k_reset, k_respawn, k_list_filter.
#include <vector>

#define ZS_DEFINE_RESET_KERNELS
#include "zs_launch.hpp"
#include "zs_reset.hpp"

hipError_t launch_reset_k(unsigned grid, size_t lds, hipStream_t s, const Dev& d, int list_mode, const int* list,
                          const int* count, const uint8_t* mask, int* err, void* obs) {
    hipLaunchKernelGGL(k_reset, dim3(grid), dim3(64), lds, s, d, list_mode, list, count, mask, err, obs);
    return hipGetLastError();
}

hipError_t launch_respawn_k(unsigned grid, size_t lds, hipStream_t s, const Dev& d) {
    hipLaunchKernelGGL(k_respawn, dim3(grid), dim3(64), lds, s, d);
    return hipGetLastError();
}

hipError_t launch_list_filter(unsigned grid, hipStream_t s, const int* src, const int* src_count, int* dst,
                              int* dst_count, const uint8_t* mask, int N) {
    hipLaunchKernelGGL(k_list_filter, dim3(grid), dim3(256), 0, s, src, src_count, dst, dst_count, mask, N);
    return hipGetLastError();
}

hipError_t reset_lds_attr(int bytes) {
    hipError_t e = hipFuncSetAttribute((const void*)k_reset, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute((const void*)k_respawn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// diagnostic builds (-DZS_STAMPS): the reset phases k_reset's workgroups stamped in this unit
hipError_t stamps_reset(unsigned long long* wg, int clear) {
#ifdef ZS_STAMPS
    const size_t nw = (size_t)ZS_STAMP_WGS * ZS_NPHASE;
    hipError_t e = hipMemcpyFromSymbol(wg, HIP_SYMBOL(g_stamp_wg), nw * sizeof(unsigned long long));
    if (e == hipSuccess && clear) {
        std::vector<unsigned long long> z(nw, 0ull);
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_wg), z.data(), nw * sizeof(unsigned long long));
    }
    return e;
#else
    (void)wg, (void)clear;
    return hipErrorNotSupported;
#endif
}
