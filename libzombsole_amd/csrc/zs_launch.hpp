// zs_launch.hpp — host launchers of the engine's kernels.
//
// The kernels are compiled in several translation units so the library builds in parallel:
//   k_tick_g.hip  once per lanes-per-env G (-DZS_G=1..64): k_tick<G, 5/6> and the fused k_step<G>
//   k_obs_t.hip   once per observation dtype (-DZS_OBS_T=0/1/2): every observation kernel
//   k_reset.hip   k_reset, k_respawn, k_list_filter
//   engine.hip    the C ABI, the layout choice and the small helper kernels
// Each unit exports plain host functions that launch its kernels; nothing but Dev, ObsLayout and
// plain pointers crosses the units.
#pragma once
#include "zs_device.hpp"

// one step launch's arguments (k_tick, or k_step when fused)
struct TickArgs {
    const int32_t* actions;
    double* rew;
    uint8_t* done;
    uint8_t* trunc;
    uint8_t* listed;
    uint8_t* reset_out;
    int* rlist;          // the pending-reset list this step appends to
    int* rcount;
    void* obs;
    int env0, env1;      // k_tick's env range
    int n_reset;         // k_step: reset-work workgroups ahead of the tick workgroups
    const int* cur_list;  // k_step: the pending list this step drains
    const int* cur_count;
    int* err;
};

#define ZS_TICK_DECL(G)                                                                                          \
    hipError_t launch_tick_g##G(int fused, int waves, unsigned grid, size_t lds, hipStream_t s, const Dev& d, \
                                const TickArgs& a);                                                            \
    hipError_t stamps_g##G(unsigned long long* wg, unsigned long long* tl, int clear);
ZS_TICK_DECL(1)
ZS_TICK_DECL(2)
ZS_TICK_DECL(4)
ZS_TICK_DECL(8)
ZS_TICK_DECL(16)
ZS_TICK_DECL(32)
ZS_TICK_DECL(64)
#undef ZS_TICK_DECL

// observation kernels
enum { OBSK_OBS = 0, OBSK_GATHER, OBSK_PIPE, OBSK_PATCH, OBSK_RING, OBSK_BRING };
struct ObsLaunch {
    int kind;         // OBSK_*
    int nobs;         // 1, 2 or 4 (k_obs: any)
    int patched;      // k_obs_ring: padded-table encoders
    unsigned grid;
    unsigned block;
    size_t lds;
    void* obs;
    const uint8_t* mask;
    ObsLayout L;
    int env0, env1;
    int stat;         // k_obs: static words staged; k_obs_gather: static words from LDS tables
    int us;           // k_obs_pbring: unit slots of the ring
};
#define ZS_OBS_DECL(T)                                                              \
    hipError_t launch_obs_##T(const ObsLaunch& o, hipStream_t s, const Dev& d); \
    hipError_t obs_lds_attr_##T(int kind, int nobs, int patched, int bytes);
ZS_OBS_DECL(i64)
ZS_OBS_DECL(i32)
ZS_OBS_DECL(i16)
#undef ZS_OBS_DECL

// reset work
hipError_t launch_reset_k(unsigned grid, size_t lds, hipStream_t s, const Dev& d, int list_mode, const int* list,
                          const int* count, const uint8_t* mask, int* err, void* obs);
hipError_t launch_respawn_k(unsigned grid, size_t lds, hipStream_t s, const Dev& d);
hipError_t launch_list_filter(unsigned grid, hipStream_t s, const int* src, const int* src_count, int* dst,
                              int* dst_count, const uint8_t* mask, int N);
hipError_t reset_lds_attr(int bytes);
hipError_t stamps_reset(unsigned long long* wg, int clear);
