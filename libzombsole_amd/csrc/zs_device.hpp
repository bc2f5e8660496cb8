// zs_device.hpp — device-side data layout and primitives of the MI355X zombsole engine.
//
// Layout in HBM (N envs, E = A + P + Z entity slots, O obstacles, W x H map, DW = ceil(W*H/32)):
//   * entity arrays, env-major [N][E] (EIX): pos (x | y << 16, int16 each), life (int32),
//     weapon (u8), present (u8), serial (u32), order (u8 dict-order list)
//       -> the lanes of an env group (one lane per slot) read one env's contiguous row: a wave of
//          4 envs x 12 slots touches 3 lines per int32 array instead of one line per slot.
//   * per-env scalars [k][N] (World.t, deaths, zombie_deaths, ...), agent tracker [a][N].
//   * env-major per-env blocks (a lane group walks its own env):
//       dead     [N][DW] u32       dead-body decoration bitmap
//       obstacle hp [N][O] int32, present / nonpos bitmaps [N][OW] u32
//       MT19937 ring [N][2][624] u32 (current block + precomputed next block)
//   * no occupancy bitmap is stored: the step / respawn kernels rebuild it in LDS from the static
//     obstacle bitmap, the env's obstacle-present bits and its things' positions.
//   * static, shared by all envs: cellmap (cell -> obstacle index), obstacle occupancy bitmap,
//     objective bitmap, obstacle xy/kind, spawn lists.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zombsole_mi355x.h"

// minimum waves per SIMD the one-wave step / tick / reset kernels are compiled for (register budget):
// 6 caps k_tick at 80 VGPRs (88 unbounded: 5 waves) for a few dwords of scratch on cold paths;
// measured C3 125 -> 127, C5 109 -> 114 M env-steps/s, C4 unchanged; 8 (64 VGPRs) spills more and
// loses at C4
#ifndef ZS_STEP_WAVES
#define ZS_STEP_WAVES 6
#endif
// The fused step launch (k_step) is chosen only when the whole launch is resident at once (at most
// 4 * ZS_FUSED_WAVES one-wave workgroups per CU), and k_reset runs a few waves per CU beside the tick
// (3.8 measured at C3): neither needs k_tick's occupancy, and at 6 waves both spill (k_step 244,
// k_reset 292 bytes of scratch per lane, on their serial chains).  3 waves: 147 / 151 VGPRs, none.
#ifndef ZS_FUSED_WAVES
#define ZS_FUSED_WAVES 3
#endif
#ifndef ZS_RESET_WAVES
#define ZS_RESET_WAVES 3
#endif

#define ZS_MT_N 624
#define ZS_MT_M 397
#define ZS_RING_WORDS (2 * ZS_MT_N)

// entity slot s of env e in the env-major entity arrays [N][E] (pos, life, weapon, present, order, serial)
#define EIX(d, s, e) ((size_t)(e) * (d).E + (s))

// per-env scalar rows
enum {
    S_T = 0,        // World.t (core.py:17)
    S_DEATHS,       // World.deaths
    S_ZD,           // World.zombie_deaths
    S_EPSTEPS,      // steps since reset (TimeLimit)
    S_NORDER,       // entities present (length of the dict-order list)
    S_NEEDRESET,    // autoreset pending
    S_PREVZD,       // reward tracker zombie_deaths (gym/reward.py:23,70)
    S_SERIAL,       // spawn serial counter (state views)
    S_ODIRTY,       // some obstacle may need removal at the next cleanup
    S_NSCAL
};

// one env's observation image in LDS (zs_obs.hpp)
struct ObsLayout {
    int win;     // window-map bytes (0: no window map, entities found by a per-cell scan)
    int off_pos, off_life, off_cw, off_dead, off_opres, off_hp;
    int hp_cap;  // obstacle HP staged in LDS (else read from HBM)
    int bytes;   // one env's image
};

__host__ __device__ inline ObsLayout obs_layout(int nobs, int plane, int E, int DW, int OW, int O, bool winmap,
                                                bool stage_hp) {
    ObsLayout L;
    int o = 0;
    L.win = winmap ? ((nobs * plane + 15) / 16) * 16 : 0;
    o += L.win;
    L.off_pos = o;
    o += E * 4;
    o = ((o + 7) / 8) * 8;  // the store-stream kernels read {code word, life} pairs from off_life as 8 B
    L.off_life = o;
    o += E * 4;
    L.off_cw = o;
    o += E * 4;
    L.off_dead = o;
    o += DW * 4;
    L.off_opres = o;
    o += OW * 4;
    L.off_hp = o;
    L.hp_cap = stage_hp ? O : 0;
    o += L.hp_cap * 4;
    L.bytes = ((o + 15) / 16) * 16;
    return L;
}

struct Dev {
    int N, W, H, O, A, P, Z, E, OW, DW, ncand, nps, nzs, nobj;
    int rw_cap;      // RNG window words staged in LDS per env (tick kernel)
    int rw_step;     // words prefetched for a plain step (resets prefetch rw_cap)
    int cand_cap;    // spawn-candidate entries staged in LDS per env (0 = global scratch)
    int lists_cap;   // static spawn-list entries staged in LDS per workgroup (0 = read from global)
    int rlists_cap;  // the same for the reset work (k_reset has its own LDS budget; = lists_cap when fused)
    int fobs;        // observations are written by the step launch itself (tick and reset work)
    int defer_respawn;  // zombie respawn left to k_respawn (wave per env) instead of the tick's leader
    int par_exec;       // the env's lanes execute the shuffled actions (zs_tick.hpp grp_execute), else its leader
    ObsLayout obsl;  // one env's observation image (zs_obs.hpp)
    int obs_stat;    // static observation tables staged beside the image (4 * DW words), 0 = none
    int rules, reward_mode, obs_scope, obs_enc, obs_w, obs_dtype, max_steps;
    int initial_zombies, minimum_zombies;
    uint32_t flags;
    // static
    const int16_t* cellmap;
    const uint32_t* obstbits;  // static obstacle occupancy bitmap [DW]
    const uint32_t* objbits;
    const int32_t* scell;      // static: per-cell obstacle index + 1 | code << 16 | objective << 20 (zs_obs.hpp)
    const uint32_t* boxbits;   // static: cell holds a Box [DW]
    const int32_t* oprefix;    // static: obstacles in cells < 32*w (obstacle index = cell rank) [DW]
    // static, k_obs_patch (zs_obs.hpp): the map padded by half a window on every side, one u16 per
    // padded cell (opad_w x opad_n / opad_w), and per obstacle its packed cell and kind (opk)
    const uint16_t* opad;
    int opad_w, opad_n;
    const uint32_t* opk;
    const int32_t* obst_xy;  // packed x | y << 16
    const uint8_t* obst_kind;
    const int32_t* pspawn;   // packed
    const int32_t* zspawn;   // packed
    const int32_t* agent_weapons;
    const int32_t* agent_codes;
    const int32_t* bot_types;
    // per env
    int32_t* pos;
    int32_t* life;
    uint8_t* weapon;
    uint8_t* present;
    uint32_t* serial;
    uint8_t* order;
    int32_t* scal;
    int32_t* prev_life;
    uint8_t* listed;
    // [N][O] int32.  The reference's obstacle life is an unbounded Python int on map objects that are
    // re-spawned at every reset with the life they had (game.py:151-155) and can be hit again before
    // the first cleanup (core.py:72-78,168-184), so it falls without a floor across episodes.  int32
    // holds it exactly down to ZS_HP_FLOOR (> 9 M episodes of maximal damage to one obstacle); below
    // that the tick saturates it and raises ZS_OVF_INT32 in *ovf (zs_overflow).
    int32_t* obst_hp;
    // [N]: bit k set once an obstacle of chunk k (obstacles k * hp_chunk .. + hp_chunk - 1) may have left
    // its MAX_LIFE (set_target_life, zs_set_state); a clean chunk's HP is hp_init's, so the observation
    // kernels read it from that shared static row (cache-resident) instead of the env's row in HBM
    uint32_t* hp_dirty;
    const int32_t* hp_init;  // [O] Box / Wall MAX_LIFE
    int hp_chunk;            // ceil(O / 32)
    uint32_t hp_chunk_m;     // ceil(2^20 / hp_chunk): o / hp_chunk = (o * hp_chunk_m) >> 20 for o < 2^16 / hp_chunk
    uint32_t hp_chunk_m32;   // ceil(2^32 / hp_chunk): o / hp_chunk = umulhi(o, hp_chunk_m32) for every o < 2^32 / hp_chunk
    // [N]: bit k set once a dead-body word of chunk k (words k * dead_chunk .. + dead_chunk - 1) may be
    // non-zero (tick cleanup, zs_set_state; k_reset clears it with the row): the prefetching observation
    // kernels read a clean chunk from dead_zero, so an env with few bodies reads few dead words
    uint32_t* dead_dirty;
    const uint32_t* dead_zero;  // [DW] zeros
    int dead_chunk;             // ceil(DW / 32)
    uint32_t dead_chunk_m;      // ceil(2^20 / dead_chunk), as hp_chunk_m
    uint32_t dead_chunk_m32;    // ceil(2^32 / dead_chunk), as hp_chunk_m32
    const uint32_t* opres_full;  // [OW] every obstacle present (the row of an env with no HP chunk dirty)
    uint32_t w_m;               // ceil(2^20 / W): c / W = (c * w_m) >> 20 for every cell c (0: not exact, divide)
    uint32_t* obst_present;
    uint32_t* obst_nonpos;
    uint32_t* dead;
    uint32_t* ring;
    uint32_t* rngst;
    // zs_step_graph: the bench policy (zs_gen_actions) is generated by the step launch itself for step
    // *pol_step with pol_n discrete actions (0: actions read from the caller's buffer)
    const uint64_t* pol_step;
    int pol_n;
    // the step's tail (zs_step), done by the last launch of the step (the observation kernel, or
    // k_tail): zero the pending-list counter this step drained and the deferred-respawn counter (the
    // next step appends to them), advance the policy step counter; null fields = nothing to do
    int* tail_cnt0;
    int* tail_cnt1;
    uint64_t* tail_step;
    uint64_t* seeds;
    int32_t* cand;
    int* resp_list;   // envs whose respawn the tick deferred to k_respawn [N]
    int* resp_count;
    // ZS_FLAG_DEATH_LOG: per env, the things its last tick's cleanup removed, {slot, serial, x, y, life}
    // each in removal order ([N][E][5]), and their count ([N]); null = not kept
    int32_t* dlog;
    int32_t* dlog_n;
    // with the death log: the actions the last tick executed, in execution order (the shuffled list of
    // core.py:76), {slot | kind << 8, target} each ([N][E][2]), and their count ([N]); the drop-in views
    // derive World.events from it (core.py:68-70, 103-119)
    int32_t* alog;
    int32_t* alog_n;
    // sticky range flags of the handle (zs_overflow): ZS_OVF_INT16 once an obstacle's life went below
    // the int16 range (int16 observations then saturate it), ZS_OVF_INT32 once one saturated at
    // ZS_HP_FLOOR (the engine then differs from the reference's unbounded int)
    uint32_t* ovf;
};

// the launch's Dev (its first kernel argument, at kernarg offset 0) through a pointer the compiler cannot
// see through, so the fields read after it are loaded where they are used instead of held in SGPRs across
// the whole kernel (tick_wg, reset_env_wave, respawn_env_wave, k_obs_ring's encoders).
// Contract: only for kernels whose FIRST argument is the Dev, unmodified (k_tick, k_step, k_reset, k_respawn,
// k_obs_ring); d0 is that argument.  -DZS_CHECK_LAUNDER builds (host-compiled check, never the product)
// compare the reloaded pointer's fields with d0 and trap on a mismatch.
__device__ __forceinline__ const Dev* zs_launder_dev(const Dev& d0) {
    typedef const __attribute__((address_space(4))) Dev CDev;
    CDev* dp = (CDev*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(dp));
#ifdef ZS_CHECK_LAUNDER
    if (dp->N != d0.N || dp->E != d0.E || dp->pos != d0.pos || dp->ring != d0.ring) __builtin_trap();
#else
    (void)d0;
#endif
    return (const Dev*)dp;
}

// lowest obstacle life the engine holds exactly; INT32_MIN itself marks an absent obstacle in the
// observation kernels' compact images (ZS_HP_ABSENT, zs_obs.hpp)
#define ZS_HP_FLOOR (-2147483647)

// an obstacle life about to be stored: saturated at ZS_HP_FLOOR (64-bit arithmetic, no wrap), range
// flags raised (rare path: one global atomic)
__device__ __forceinline__ int32_t hp_store_value(const Dev& d, int64_t v) {
    if (v < -32768) {
        uint32_t f = ZS_OVF_INT16;
        if (v < (int64_t)ZS_HP_FLOOR) {
            v = ZS_HP_FLOOR;
            f |= ZS_OVF_INT32;
        }
        // one flag word for the handle: skip the atomic once the flags are up (every later hit would
        // otherwise contend for this address)
        if ((__hip_atomic_load(d.ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & f) != f) atomicOr(d.ovf, f);
    }
    return (int32_t)v;
}

// the step's tail (see Dev::tail_*), by one thread of the last launch of a zs_step
__device__ __forceinline__ void step_tail(const Dev& d) {
    if (d.tail_cnt0) *d.tail_cnt0 = 0;
    if (d.tail_cnt1) *d.tail_cnt1 = 0;
    if (d.tail_step) *d.tail_step += 1;
}

// bench / parity action stream (libzombsole_amd/actions.py): agent a of env e at step t takes
// DISCRETE[splitmix64(splitmix64(splitmix64(seed_e) ^ t) ^ a) % n]
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static __constant__ int32_t c_discrete[7][3] = {{ZS_ACT_MOVE, 0, 1},  {ZS_ACT_MOVE, -1, 0},       {ZS_ACT_MOVE, 0, -1},
                                         {ZS_ACT_MOVE, 1, 0},  {ZS_ACT_ATTACK_CLOSEST, 0, 0}, {ZS_ACT_HEAL, 0, 0},
                                         {ZS_ACT_HEAL_CLOSEST, 0, 0}};

// the policy's discrete action id for agent a of the env seeded `seed`
__device__ __forceinline__ int policy_id(uint64_t seed, uint64_t step, int n, int a) {
    return (int)(splitmix64(splitmix64(splitmix64(seed) ^ step) ^ (uint64_t)a) % (uint64_t)n);
}
// component k (0..3A) of an env's action triples under the policy
__device__ __forceinline__ int32_t policy_action(uint64_t seed, uint64_t step, int n, int k) {
    const int a = k / 3;
    return c_discrete[policy_id(seed, step, n, a)][k - 3 * a];
}

__device__ __forceinline__ int32_t pack_xy(int x, int y) { return (int32_t)((uint32_t)(x & 0xffff) | ((uint32_t)y << 16)); }
__device__ __forceinline__ int unpack_x(int32_t p) { return (int)(int16_t)(p & 0xffff); }
__device__ __forceinline__ int unpack_y(int32_t p) { return (int)(p >> 16); }

// ---------------------------------------------------------------------------
// CPython MT19937 stream, one per env.
// The ring holds two consecutive 624-word blocks of the raw (untempered) MT
// sequence x[k]: the block being consumed and, when `ready`, the next one, so a
// lane can draw >= 624 words without twisting.  x[k+624] = x[k+397] ^ f(x[k], x[k+1])
// lets the next block be produced from the current one (serially in a lane on
// the rare slow path, cooperatively by a whole wave in zs_rng_refill).
// rngst packs: offset (bits 0..9), current slot (bit 10), next-ready (bit 11).
// ---------------------------------------------------------------------------
// Lane hand-off through LDS inside a one-wave workgroup.  LDS instructions of a wave execute in
// program order, so lanes only need the compiler kept from reordering across this point; unlike
// __syncthreads() (a workgroup release fence) it does not wait for outstanding global stores.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_f(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// dst = the 624-word block that follows src (Modules/_randommodule.c genrand_uint32 twist)
__device__ inline void mt_twist_serial(uint32_t* dst, const uint32_t* src) {
    for (int i = 0; i < ZS_MT_N; i++) {
        uint32_t b = (i + 1 < ZS_MT_N) ? src[i + 1] : dst[0];
        uint32_t c = (i + ZS_MT_M < ZS_MT_N) ? src[i + ZS_MT_M] : dst[i + ZS_MT_M - ZS_MT_N];
        dst[i] = mt_f(src[i], b, c);
    }
}

__device__ __forceinline__ uint32_t st_pack(uint32_t off, uint32_t slot, uint32_t ready) {
    return off | (slot << 10) | (ready << 11);
}

// ring state after consuming n more words from st (n <= 624; when the words cross into the
// other slot that slot held the next block, i.e. st was `ready`)
__device__ __forceinline__ uint32_t st_advance(uint32_t st, uint32_t n) {
    uint32_t off = (st & 1023u) + n, slot = (st >> 10) & 1u, ready = (st >> 11) & 1u;
    if (off > ZS_MT_N) {
        slot ^= 1u;
        off -= ZS_MT_N;
        ready = 0;
    }
    return st_pack(off, slot, ready);
}

// ---------------------------------------------------------------------------
// weapons (weapons.py:18-25) with the sqrt range tests as exact integer d^2
// bounds: dist > 1.5 <=> d2 >= 3, > 3 <=> d2 >= 10, > 6 <=> d2 >= 37, > 10 <=> d2 >= 101
// ---------------------------------------------------------------------------
__device__ __forceinline__ int weapon_r2(int w) {
    return w == ZS_WEAPON_GUN ? 36 : w == ZS_WEAPON_RIFLE ? 100 : w == ZS_WEAPON_SHOTGUN ? 9 : 2;
}
__device__ __forceinline__ int weapon_lo(int w) {
    return w == ZS_WEAPON_AXE ? 75 : w == ZS_WEAPON_GUN ? 10 : w == ZS_WEAPON_RIFLE ? 25 : w == ZS_WEAPON_SHOTGUN ? 75 : 5;
}
__device__ __forceinline__ int weapon_hi(int w) {
    return w == ZS_WEAPON_AXE ? 100 : w == ZS_WEAPON_GUN ? 50 : w == ZS_WEAPON_RIFLE ? 75 : w == ZS_WEAPON_SHOTGUN ? 100 : 10;
}

__device__ __forceinline__ int d2(int x1, int y1, int x2, int y2) {
    int dx = x1 - x2, dy = y1 - y2;
    return dx * dx + dy * dy;
}

// d2 of two packed positions (pack_xy) whose coordinate differences fit int16 (two cells of a map): one
// packed int16 subtract and one int16 dot product
typedef short zs_v2s __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int d2p(int32_t a, int32_t b) {
    const zs_v2s v = __builtin_bit_cast(zs_v2s, a) - __builtin_bit_cast(zs_v2s, b);
    return __builtin_amdgcn_sdot2(v, v, 0, false);
}

__device__ __forceinline__ int64_t floordiv100(int64_t a) {  // Python a // 100
    int64_t q = a / 100;
    if ((a % 100) != 0 && a < 0) q -= 1;
    return q;
}

// Explicit LDS (address space 3) pointer types for every view into the workgroup's image, so the
// compiler always emits ds_* instructions (a pointer that might be LDS or global degrades to
// flat accesses and pushes the lane context to scratch).
#define ZS_LDS __attribute__((address_space(3)))
typedef ZS_LDS uint32_t lu32;
typedef ZS_LDS int32_t li32;
typedef ZS_LDS uint16_t lu16;
typedef ZS_LDS uint8_t lu8;

// One wave twists the 624-word block src into nw (both LDS; _randommodule.c genrand_uint32), in the
// three dependency phases of the in-place update (words [0, 227) from src alone, [227, 454) reading
// phase 1's new words, [454, 624) phase 2's and nw[0]).  Each phase's reads are issued before its
// stores (no read of a phase touches a word it writes): one LDS round trip per phase, not one per word
// group.  The caller syncs the wave before (src complete) and after (nw complete).
__device__ __forceinline__ void lds_twist(const ZS_LDS uint32_t* src, ZS_LDS uint32_t* nw, int lane) {
    constexpr int N = ZS_MT_N, M = ZS_MT_M, P1 = N - M, P3 = N - 2 * P1, K1 = (P1 + 63) / 64, K3 = (P3 + 63) / 64;
    static_assert(P3 > 0 && P3 <= P1, "MT19937 phase split");
    uint32_t a[K1], b[K1], c[K1];
#pragma unroll
    for (int u = 0; u < K1; u++) {
        const int k = min(lane + 64 * u, P1 - 1);
        a[u] = src[k];
        b[u] = src[k + 1];
        c[u] = src[k + M];
    }
#pragma unroll
    for (int u = 0; u < K1; u++)
        if (lane + 64 * u < P1) nw[lane + 64 * u] = mt_f(a[u], b[u], c[u]);
    wave_sync();
#pragma unroll
    for (int u = 0; u < K1; u++) {
        const int k = P1 + min(lane + 64 * u, P1 - 1);
        a[u] = src[k];
        b[u] = src[k + 1];
        c[u] = nw[k + M - N];
    }
#pragma unroll
    for (int u = 0; u < K1; u++)
        if (lane + 64 * u < P1) nw[P1 + lane + 64 * u] = mt_f(a[u], b[u], c[u]);
    wave_sync();
#pragma unroll
    for (int u = 0; u < K3; u++) {
        const int k = 2 * P1 + min(lane + 64 * u, P3 - 1);
        a[u] = src[k];
        b[u] = k + 1 < N ? src[k + 1] : nw[0];
        c[u] = nw[k + M - N];
    }
#pragma unroll
    for (int u = 0; u < K3; u++)
        if (lane + 64 * u < P3) nw[2 * P1 + lane + 64 * u] = mt_f(a[u], b[u], c[u]);
}

// Stage n global words into LDS: lane `lane0` of a team of `step` lanes copies elements
// lane0, lane0 + step, ...  All loads of a chunk of 8 are issued before any LDS store, so one
// memory latency is paid per chunk instead of one per element.
template <typename T, typename LT, typename Idx>
__device__ __forceinline__ void stage_in(const T* src, int n, int lane0, int step, LT* dst, Idx dst_index) {
    for (int b = lane0; b < n; b += 8 * step) {
        T v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            int i = b + u * step;
            v[u] = src[i < n ? i : n - 1];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            int i = b + u * step;
            if (i < n) dst[dst_index(i)] = v[u];
        }
    }
}
