// k_tick_g.hip — the step kernels for one lanes-per-env count G (compiled once per G, -DZS_G=G):
// k_tick<G, 5/6> (the tick alone, zs_tick.hpp) and k_step<G> (reset work + tick in one launch).
#include <vector>

#include "zs_launch.hpp"
#include "zs_reset.hpp"

#ifndef ZS_G
#error "compile with -DZS_G=<lanes per env>"
#endif

// One launch per step: workgroups [0, n_reset) rebuild the envs of the pending list (next-step
// autoreset, World rebuilt as in game.py:151-169), the others tick every other env (zs_tick.hpp).
// An env is either pending (reset work only; the tick reports it as reset without touching its
// state) or stepping (tick only), so the two roles never share an env.
// Dev is the first argument: tick_wg / reset_env_wave reload it from kernarg offset 0 (zs_launder_dev)
template <int G>
__global__ void __launch_bounds__(64, ZS_FUSED_WAVES) k_step(Dev d, int n_reset, const int32_t* actions, double* rew,
                                             uint8_t* done_out, uint8_t* trunc_out, uint8_t* listed_out,
                                             uint8_t* reset_out, int* reset_list, int* reset_count,
                                             const int* cur_list, const int* cur_count, int* err_out, void* obs_out) {
    extern __shared__ __align__(16) uint8_t smem[];
    TL(0);
    if ((int)blockIdx.x < n_reset)
        reset_role(d, 1, cur_list, cur_count, nullptr, err_out, blockIdx.x, n_reset, d.fobs ? obs_out : nullptr);
    else
        tick_wg<G, true>(d, xcd_remap(blockIdx.x - n_reset, gridDim.x - n_reset), actions, rew, done_out, trunc_out,
                   listed_out, reset_out, reset_list, reset_count, obs_out, 0, d.N, (lu8*)smem);
    TL(1);
}

#define ZS_CAT2(a, b) a##b
#define ZS_CAT(a, b) ZS_CAT2(a, b)

hipError_t ZS_CAT(launch_tick_g, ZS_G)(int fused, int waves, unsigned grid, size_t lds, hipStream_t s, const Dev& d,
                                       const TickArgs& a) {
    constexpr int G = ZS_G;
    if (fused)
        hipLaunchKernelGGL(k_step<G>, dim3(grid + a.n_reset), dim3(64), lds, s, d, a.n_reset, a.actions, a.rew, a.done,
                           a.trunc, a.listed, a.reset_out, a.rlist, a.rcount, a.cur_list, a.cur_count, a.err, a.obs);
    else if (waves == 5)
        hipLaunchKernelGGL((k_tick<G, 5>), dim3(grid), dim3(64), lds, s, d, a.actions, a.rew, a.done, a.trunc, a.listed,
                           a.reset_out, a.rlist, a.rcount, a.obs, a.env0, a.env1);
    else
        hipLaunchKernelGGL((k_tick<G, 6>), dim3(grid), dim3(64), lds, s, d, a.actions, a.rew, a.done, a.trunc, a.listed,
                           a.reset_out, a.rlist, a.rcount, a.obs, a.env0, a.env1);
    return hipGetLastError();
}

// diagnostic builds (-DZS_STAMPS): this unit's per-phase sums and the step launch's timeline
hipError_t ZS_CAT(stamps_g, ZS_G)(unsigned long long* wg, unsigned long long* tl, int clear) {
#ifdef ZS_STAMPS
    const size_t nw = (size_t)ZS_STAMP_WGS * ZS_NPHASE;
    hipError_t e = hipSuccess;
    if (wg) e = hipMemcpyFromSymbol(wg, HIP_SYMBOL(g_stamp_wg), nw * sizeof(unsigned long long));
    if (e == hipSuccess && tl) e = hipMemcpyFromSymbol(tl, HIP_SYMBOL(g_stamp_tl), (size_t)ZS_STAMP_WGS * 2 * sizeof(unsigned long long));
    if (e == hipSuccess && clear) {
        std::vector<unsigned long long> z(nw, 0ull);
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_wg), z.data(), nw * sizeof(unsigned long long));
    }
    return e;
#else
    (void)wg, (void)tl, (void)clear;
    return hipErrorNotSupported;
#endif
}
