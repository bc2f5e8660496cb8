// zs_fstep.hpp — k_fstep: one step (reset work, tick and observations) as one persistent launch whose
// workgroups overlap the tick with the observation stream inside the step.
//
// The unfused step runs k_tick (issue / latency bound: C3 86 us), then k_obs_ring (HBM-write bound:
// C3 266 us) back to back, so the step costs their sum.  Envs are independent, so the observations of
// env block b can stream while block b + 1 ticks.  One workgroup per CU owns a contiguous range of the
// step's tick units (64 / G envs each) and splits its waves into three roles:
//   * NT tick waves take the range's units from an LDS counter and run the tick on each
//     (tick_wg, zs_tick.hpp: decisions, shuffle, execution, cleanup, rewards, rules for the stepping
//     envs; gym/multiagent_env.py:111-171 with core.py:72-78), then rebuild the unit's envs that ended
//     at the previous step (reset_env_wave, zs_reset.hpp; game.py:151-169: the next-step autoreset the
//     unfused step leaves to k_reset on its side stream), and publish the unit as ready in LDS;
//   * NEN encoder waves walk the range's envs in order, wait for each env's unit, load the env's new
//     state (its dirty masks from LDS, where the tick wave published them) and encode its agents'
//     21 x 21 x 3 windows into a ring slot with the
//     padded-table encoder (PatchEnc, zs_obs.hpp; gym/observation.py:57-173), the next env's loads in
//     flight while one env encodes;
//   * NW writer waves stream the ring's slots out as 16-B stores (obs_stage_flush), as k_obs_ring's do.
// No wave waits on a wave of another workgroup, and inside the workgroup the waits only point from
// encoders to tick waves (a unit is published once ticked) and to writers (a slot is free once written
// out), writers to encoders (a slot is written out once filled), all in rising order: every wave reaches
// its end.  The last workgroup to finish does the step's tail (Dev::tail_*): the pending list this step
// drained by flag (S_NEEDRESET) is emptied and the policy's step counter advanced.
#pragma once
#include "zs_obs.hpp"
#include "zs_reset.hpp"
#include "zs_tick.hpp"
#include "zs_launch.hpp"

// device-scope loads: the dirty masks, which the tick updates with device-scope atomics and 16 envs share
// a cache line of (a line another wave of this CU loaded earlier may be in its L1)
template <typename V>
__device__ __forceinline__ V ld_dev(const V* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// obs_prefetch_env's loads (zs_obs.hpp) for env e with its dirty masks dq (published in LDS by the tick
// wave): the entity slots, dead-body words, present words and obstacle HP.  Plain loads: the tick wave that
// wrote them is in this workgroup and released them before publishing the env (a workgroup-scope release /
// acquire pair needs no cache maintenance on gfx950: the CU's waves share its L1).
__device__ __forceinline__ void fs_prefetch_env(const Dev& d, int e, zs_v2u dq, ObsPrefetch& f) {
    const int lane = threadIdx.x & 63;
    const uint32_t hd = dq.x, dd = dq.y;
    const int s = lane < d.E ? lane : d.E - 1;
    f.pos = d.pos[EIX(d, s, e)];
    f.life = d.life[EIX(d, s, e)];
    f.wp = d.weapon[EIX(d, s, e)];
    f.pr = d.present[EIX(d, s, e)];
    const uint32_t* dr = d.dead + (size_t)e * d.DW;
#pragma unroll
    for (int i = 0; i < OBS_PF_D; i++) {
        const int w = min(lane + 64 * i, d.DW - 1);
        f.dead[i] = (((dd >> ((w * d.dead_chunk_m) >> 20)) & 1u) ? dr : d.dead_zero)[w];
    }
    f.opres = (hd ? d.obst_present + (size_t)e * d.OW : d.opres_full)[min(lane, max(d.OW - 1, 0))];
    const int32_t* hr = d.obst_hp + (size_t)e * d.O;
#pragma unroll
    for (int i = 0; i < OBS_PF_H; i++) {
        const int o = min(lane + 64 * i, d.O - 1);
        f.hp[i] = (((hd >> ((o * d.hp_chunk_m) >> 20)) & 1u) ? hr : d.hp_init)[o];
    }
}

// EARLY: the tick's RNG window loaded with its first load round (tick_wg; the one-round shapes, where each
// tick wave takes one unit and the window's round trip is on the step's critical path)
template <int G, typename T, int NOBS, int NT, int NEN, int NW, bool EARLY = false>
__global__ void __launch_bounds__(64 * (NT + NEN + NW), 1) k_fstep(Dev d, FsArgs a) {
    extern __shared__ __align__(16) uint8_t smem[];
    typedef typename obs_stage<T>::type S;
    constexpr int NE = 64 / G, WW = 21, PLANE = WW * WW, TS = (int)sizeof(T);
    constexpr int PAIR = ring_pair(TS, NOBS), BLK = NOBS * 3 * PLANE;
    const FsLayout& FL = a.L;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // this workgroup's tick units [u0, u1) and envs [e_lo, e_lo + n_env)
    const int nunits = (d.N + NE - 1) / NE;
    const int upw = (nunits + (int)gridDim.x - 1) / (int)gridDim.x;
    const int u0 = min((int)blockIdx.x * upw, nunits), u1 = min(u0 + upw, nunits), nu = u1 - u0;
    const int e_lo = u0 * NE, n_env = max(0, min(u1 * NE, d.N) - e_lo);
    ZS_LDS int* state = (ZS_LDS int*)(smem + FL.off_state);  // ring protocol word per slot and env of a unit
    ZS_LDS int* ready = (ZS_LDS int*)(smem + FL.off_ready);  // 1 once tick unit u0 + k is ticked and reset
    ZS_LDS int* ctr = (ZS_LDS int*)(smem + FL.off_ctr);      // next tick unit to take
    ZS_LDS zs_v2u* dqs = (ZS_LDS zs_v2u*)(smem + FL.off_dq); // {hp_dirty, dead_dirty} of env e_lo + t
    for (int i = threadIdx.x; i < 16 + FS_MAX_UNITS + 4; i += blockDim.x) state[i] = 0;  // the three arrays are adjacent
    patch_stage_static(d, smem);  // barriers: the zeroed words and the tables before any role starts
    const int US = FL.us;
    lu8* slots = (lu8*)(smem + FL.off_slots);
    if (wave < NT) {
        // ---- tick role ----
        lu8* reg = (lu8*)(smem + FL.off_tick + wave * FL.tick_bytes);
        for (;;) {
            int k = 0;
            if (lane == 0) k = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
            if (k >= nu) break;
            unsigned long long pend = 0ull;
            // the tick reads the Dev fields through a kernarg pointer the loop cannot see through, so they are
            // loaded where each unit uses them instead of being hoisted out of the loop and kept live across
            // every unit (SGPR pressure: 668 B of spills per lane)
            typedef const __attribute__((address_space(4))) Dev CDev;
            CDev* dp = (CDev*)__builtin_amdgcn_kernarg_segment_ptr();
            asm volatile("" : "+s"(dp));
            const Dev& dd = *(const Dev*)dp;
            tick_wg<G, EARLY>(dd, u0 + k, a.actions, a.rew, a.done, a.trunc, a.listed, a.reset_out, a.rlist, a.rcount, nullptr,
                       0, d.N, reg, &pend);
            wave_sync();
            if (pend) {  // the unit's envs that ended at the previous step: World rebuilt (game.py:151-169)
                const ResetLds Lr = reset_lds_carve(dd, (uint8_t*)reg);
                while (pend) {
                    const int g = (__ffsll((long long)pend) - 1) / G;
                    pend &= ~(1ull << (g * G));
                    reset_env_wave(dd, Lr, (u0 + k) * NE + g, 1, a.err);
                }
            }
            // the unit's dirty masks for its encoders (after every atomic of the unit: the loads wait for them)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane < NE && (u0 + k) * NE + lane < d.N) {
                const int e = (u0 + k) * NE + lane;
                dqs[e - e_lo] = zs_v2u{ld_dev(d.hp_dirty + e), ld_dev(d.dead_dirty + e)};
            }
            // the unit's stores completed before its flag: a workgroup release waits for them
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) ring_state_store(&ready[k], 1);
            wave_sync();
        }
    } else if (wave < NT + NEN) {
        // ---- encoder role: envs e_lo + w, + NEN, ...; the next env's loads in flight while this one encodes ----
        const int w = wave - NT;
        lu8* wb = (lu8*)(smem + FL.off_enc + w * FL.enc_bytes);
        PatchEnc<S> pe(d, smem, wb, lane);
        T* out = (T*)a.obs;
        ObsPrefetch f;
        auto fetch = [&](int t) {  // wait for env e_lo + t's unit, then issue its loads into f
            ring_wait(&ready[t / NE], 1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            fs_prefetch_env(d, e_lo + t, dqs[t], f);
        };
        if (w < n_env) fetch(w);
        for (int t = w; t < n_env; t += NEN) {
            const int e = e_lo + t;
            pe.build(d, f);
            if (t + NEN < n_env) fetch(t + NEN);
            const int u = t / PAIR, h = t % PAIR, q = u % US;
            if (u >= US) ring_wait(&state[PAIR * q + h], 2 * (u - US) + 2);
            wave_sync();
            ZS_LDS S* ot0 = (ZS_LDS S*)(slots + q * FL.slot_bytes) + (int)((uintptr_t)(out + (size_t)(e - h) * BLK) & 15) / TS +
                            h * BLK;
#pragma unroll
            for (int ag = 0; ag < NOBS; ag++) pe.block(d, ot0 + ag * 3 * PLANE, ag);
            ring_state_store(&state[PAIR * q + h], 2 * u + 1);
        }
    } else {
        // ---- writer role: ring units w, w + NW, ... (PAIR envs each) ----
        T* out = (T*)a.obs;
        const int nru = (n_env + PAIR - 1) / PAIR;
        for (int u = wave - NT - NEN; u < nru; u += NW) {
            const int q = u % US, e = e_lo + PAIR * u;
            const bool whole = PAIR * u + PAIR <= n_env;
            for (int h = 0; h < PAIR; h++)
                if (PAIR * u + h < n_env) ring_wait(&state[PAIR * q + h], 2 * u + 1);
            if (whole) obs_stage_flush<T, NOBS * PAIR, RING_THR>(slots + q * FL.slot_bytes, out + (size_t)e * BLK, lane);
            else obs_stage_flush<T, NOBS, RING_THR>(slots + q * FL.slot_bytes, out + (size_t)e * BLK, lane);
            for (int h = 0; h < PAIR; h++) ring_state_store(&state[PAIR * q + h], 2 * u + 2);
        }
    }
    // the step's tail, by the last workgroup to get here (every tick of the launch has read the policy's
    // step counter by then)
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const int k = atomicAdd(a.done_ctr, 1);
        if (k == (int)gridDim.x - 1) {
            step_tail(d);
            *a.done_ctr = 0;
        }
    }
}
