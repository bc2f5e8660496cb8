// zs_tick.hpp — the step kernel (k_tick): one env per group of G lanes, state staged in LDS.
//
// A tick of the reference is strictly sequential per env (World.step, core.py:72-78: decide
// in dict order -> random.shuffle -> execute one by one -> clean dead things), followed by the
// env glue (rewards, zombie respawn, rules).  Mapping to CDNA4:
//   * a 64-lane wave holds NE = 64/G envs; every env's hot state sits in LDS for the whole
//     tick: occupancy bitmap (1 bit per cell, rebuilt at stage-in from the static obstacle cells, the
//     env's obstacle-present bits and its things: never stored), entity table, dict-order list, a window of
//     pre-tempered MT19937 words and the spawn-candidate list, so the serial chain issues no
//     dependent global loads;
//   * the G lanes of an env stage state in/out and take the decisions in parallel (every
//     decision reads start-of-tick state only; the few RNG-consuming ones — wandering zombies,
//     hamster, randoman — are deferred to the leader and taken in dict order);
//   * the leader lane runs the order-dependent part: shuffle, execution, cleanup, rewards,
//     respawn, rules;
//   * at the end the wave twists, cooperatively, the next MT block of every env that crossed one.
// The sqrt range tests of the reference are replaced by exact integer d^2 tests.
#pragma once
#include "zs_device.hpp"
#include "zs_obs.hpp"

#define NOTHING ((int)0x80000000)

enum { K_NONE = 0, K_MOVE = 1, K_ATTACK = 2, K_HEAL = 3, K_DEFER = 4, K_RAISE = 5 };

// Diagnostic build only (-DZS_STAMPS, never the product .so): lane 0 of every workgroup adds the
// s_memtime ticks each k_tick phase took into its own slot g_stamp_wg[block][phase] (plain
// stores, no contended atomics); zs_debug_stamps sums / maxes the slots on the host.
#ifdef ZS_STAMPS
#define ZS_NPHASE 28
#define ZS_STAMP_WGS 65536
static __device__ unsigned long long g_stamp_wg[ZS_STAMP_WGS * ZS_NPHASE];
#define STAMP_DECL unsigned long long _st_prev = 0;
#define STAMP(k)                                                                          \
    do {                                                                                  \
        unsigned long long _t;                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");      \
        if ((k) > 0 && threadIdx.x == 0 && blockIdx.x < ZS_STAMP_WGS)                     \
            g_stamp_wg[blockIdx.x * ZS_NPHASE + (k)-1] += _t - _st_prev;                  \
        _st_prev = _t;                                                                    \
    } while (0)
#define SUB_DECL unsigned long long _sub_prev;
#define SUB(k)                                                                            \
    do {                                                                                  \
        unsigned long long _t;                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");      \
        if ((k) > 0 && blockIdx.x < ZS_STAMP_WGS && c.g == 0)                             \
            g_stamp_wg[blockIdx.x * ZS_NPHASE + 7 + (k)-1] += _t - _sub_prev;             \
        _sub_prev = _t;                                                                   \
    } while (0)
// stage-in splits: SX(1) after the first load round, SX(2) after the RNG window (slots 11, 12)
#define SX(k)                                                                             \
    do {                                                                                  \
        unsigned long long _t;                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");      \
        if (threadIdx.x == 0 && blockIdx.x < ZS_STAMP_WGS)                                \
            g_stamp_wg[blockIdx.x * ZS_NPHASE + 10 + (k)] += _t - _st_prev;                \
    } while (0)
#define RST_DECL unsigned long long _r_prev;
#define RST(k)                                                                            \
    do {                                                                                  \
        unsigned long long _t;                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");      \
        if ((k) > 0 && blockIdx.x < ZS_STAMP_WGS && threadIdx.x == 0)                     \
            g_stamp_wg[blockIdx.x * ZS_NPHASE + 13 + (k)-1] += _t - _r_prev;              \
        _r_prev = _t;                                                                     \
    } while (0)
// grp_execute splits (slots 20..26), lane 0 of the workgroup
#define GX_DECL unsigned long long _g_prev;
#define GX(k)                                                                             \
    do {                                                                                  \
        unsigned long long _t;                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");      \
        if ((k) > 0 && threadIdx.x == 0 && blockIdx.x < ZS_STAMP_WGS)                     \
            g_stamp_wg[blockIdx.x * ZS_NPHASE + 19 + (k)] += _t - _g_prev;                \
        _g_prev = _t;                                                                     \
    } while (0)
// slot 27: envs of the workgroup whose actions the leader executed (serial path or window fallback)
#define XEV(k) atomicAdd(&g_stamp_wg[blockIdx.x * ZS_NPHASE + 27], (unsigned long long)(k))
// workgroup timeline of the last launch: s_memrealtime (100 MHz, one clock for the whole chip) at
// the workgroup's start and end, g_stamp_tl[block][0 / 1]
static __device__ unsigned long long g_stamp_tl[ZS_STAMP_WGS * 2];
#define TL(k)                                                                             \
    do {                                                                                  \
        unsigned long long _t;                                                            \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");  \
        if (threadIdx.x == 0 && blockIdx.x < ZS_STAMP_WGS) g_stamp_tl[blockIdx.x * 2 + (k)] = _t; \
    } while (0)
#else
#define TL(k)
#define XEV(k)
#define GX_DECL
#define GX(k)
#define SX(k)
#define STAMP_DECL
#define STAMP(k)
#define SUB_DECL
#define SUB(k)
#define RST_DECL
#define RST(k)
#endif

// adjacent_positions order (utils.py:34-44)
static __constant__ int c_adj_dx[4] = {0, 0, 1, -1};
static __constant__ int c_adj_dy[4] = {1, -1, 0, 0};

// LDS footprint of one workgroup (host and device agree on this layout).  The entity columns the
// observations need (pos, life, weapon, present) sit before `region`; everything in `region` is
// dead once the tick's state is stored, so the observation image of the env being encoded and the
// MT twist buffer alias it.
struct TickLayout {
    int ne;                                  // envs per workgroup
    int off_lists;                           // static spawn lists (player then zombie), shared by the WG
    int off_misc;                            // per-env scalars / tracker, [MISC_*][ne] int32
    int off_lst;
    int off_pos, off_life, off_weap, off_pres;
    int off_region;                          // = off_bm
    int off_bm, off_rw, off_cand, off_tgt, off_act, off_order, off_rank, off_kind, off_perm, off_moved, off_xs;
    int bytes;
};

// per-env LDS scalars (MISC rows); rows MISC_N.. hold prev_life[A] then listed[A].  MISC_NMOVED and
// MISC_NORD are scratch rows of the tick's leader / group hand-off (not staged from or to HBM).
enum { MISC_T = 0, MISC_DEATHS, MISC_ZD, MISC_EPSTEPS, MISC_PREVZD, MISC_SERIAL, MISC_ODIRTY, MISC_NMOVED, MISC_NORD, MISC_N };

__host__ __device__ inline TickLayout tick_layout(int ne, int E, int DW, int rw_cap, int cand_cap, int lists_cap,
                                                  int A, int obs_bytes = 0) {
    TickLayout L;
    L.ne = ne;
    int o = 0;
    L.off_lists = o;
    o += lists_cap * 4;
    L.off_misc = o;
    o += (MISC_N + 2 * A) * ne * 4;
    L.off_lst = o;
    o += ne * 4;
    L.off_pos = o;
    o += E * ne * 4;
    L.off_life = o;
    o += E * ne * 4;
    L.off_weap = o;
    o += E * ne;
    L.off_pres = o;
    o += E * ne;
    L.off_order = o;  // the dict order is stored out after the MT refill, whose buffer aliases the region
    o += E * ne;
    o = ((o + 15) / 16) * 16;
    const int region = o;
    L.off_region = L.off_bm = o;
    o += DW * ne * 4;
    L.off_rw = o;
    o += rw_cap * ne * 4;
    L.off_tgt = o;
    o += E * ne * 4;
    L.off_act = o;  // the agents' action triples, loaded with the stage-in round
    o += 3 * A * ne * 4;
    L.off_cand = o;
    o += ((cand_cap * ne * 2 + 3) / 4) * 4;
    L.off_rank = o;
    o += E * ne;
    L.off_kind = o;
    o += E * ne;
    L.off_perm = o;
    o += E * ne;
    L.off_moved = o;
    o += E * ne;
    o = ((o + 15) / 16) * 16;
    L.off_xs = o;  // grp_execute's two tables of 64 words (G per env)
    o += 2 * 64 * 4;
    // the MT twist buffer (2 x 624 words) and one env's observation image alias the region
    if (o - region < 2 * ZS_MT_N * 4) o = region + 2 * ZS_MT_N * 4;
    if (o - region < obs_bytes) o = region + obs_bytes;
    L.bytes = o;
    return L;
}

// one env as seen by one lane of its group
struct Grp {
    int e, g, j, ne;
    li32* lists;  // static spawn lists (player then zombie) when d.lists_cap
    li32* misc;
    lu32* bm;
    lu32* rw;
    lu16* cand;
    li32* lpos;
    li32* llife;
    li32* ltgt;
    lu8* lweap;
    lu8* lpres;
    lu8* lorder;
    lu8* lrank;
    lu8* lkind;
    lu8* lperm;
    lu8* lmoved;
    li32* lact;  // agent a's action triple at 3a..3a+2
    li32* xs;    // grp_execute's tables: table k of this env at xs + 64 k + g G
    // leader registers
    uint32_t st0;  // ring state at the start of the LDS window
    int wpos, wlen;
    int n_order, t, deaths, zd, epsteps, prevzd, serial, odirty;
    int respawn;  // the zombie respawn of this step is deferred to k_respawn
    int fin;      // this step ended the episode (done or truncated)
};

#define IX(c, k) ((k) * (c).ne + (c).g)
#define LP(c, s) (c).lpos[IX(c, s)]
#define LL(c, s) (c).llife[IX(c, s)]
#define LT(c, s) (c).ltgt[IX(c, s)]
#define LW(c, s) (c).lweap[IX(c, s)]
#define LPR(c, s) (c).lpres[IX(c, s)]
#define LO(c, s) (c).lorder[IX(c, s)]
#define LR(c, s) (c).lrank[IX(c, s)]
#define LK(c, s) (c).lkind[IX(c, s)]
#define LPE(c, s) (c).lperm[IX(c, s)]
#define LM(c, s) (c).lmoved[IX(c, s)]
#define MISC(c, f) (c).misc[IX(c, f)]
#define LACT(c, k) (c).lact[IX(c, k)]

// ---------------------------------------------------------------------------
// RNG: the leader draws pre-tempered words from the LDS window; when it runs dry it reloads
// the next rw_step words (the window size; rw_cap is only the LDS capacity) from the ring by itself
// (twisting serially if the ring is behind).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void rng_reload(const Dev& d, Grp& c) {
    uint32_t st = st_advance(c.st0, c.wlen);
    uint32_t off = st & 1023u, slot = (st >> 10) & 1u, ready = (st >> 11) & 1u;
    uint32_t* ring = d.ring + (size_t)c.e * ZS_RING_WORDS;
    if (off >= ZS_MT_N) {
        if (!ready) {
            mt_twist_serial(ring + (slot ^ 1u) * ZS_MT_N, ring + slot * ZS_MT_N);
            __threadfence();  // the block's stores before any later read of it (coop_refill's loads)
        }
        slot ^= 1u;
        off = 0;
        ready = 0;
    }
    int n = d.rw_step;  // a multiple of 4 (32 .. 512)
    if ((int)off + n > ZS_MT_N && !ready) {
        mt_twist_serial(ring + (slot ^ 1u) * ZS_MT_N, ring + slot * ZS_MT_N);
        __threadfence();
        ready = 1;
    }
    for (int i0 = 0; i0 < n; i0 += 4) {  // 4 loads in flight (a wider batch costs every caller registers)
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            uint32_t q = off + i0 + u;
            v[u] = q < ZS_MT_N ? ring[slot * ZS_MT_N + q] : ring[(slot ^ 1u) * ZS_MT_N + q - ZS_MT_N];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) c.rw[IX(c, i0 + u)] = mt_temper(v[u]);
    }
    c.st0 = st_pack(off, slot, ready);
    c.wpos = 0;
    c.wlen = n;
}

__device__ __forceinline__ uint32_t rng_u32(const Dev& d, Grp& c) {
    if (c.wpos >= c.wlen) rng_reload(d, c);
    return c.rw[IX(c, c.wpos++)];
}

// Random._randbelow_with_getrandbits (random.py:239-249); getrandbits(k<=32) = u32 >> (32-k)
__device__ __forceinline__ int rng_below(const Dev& d, Grp& c, int n) {
    if (n <= 0) return 0;
    int k = 32 - __clz(n);
    uint32_t v;
    do {
        v = rng_u32(d, c) >> (32 - k);
    } while (v >= (uint32_t)n);
    return (int)v;
}

// randint(a, b) (random.py:366-370)
__device__ __forceinline__ int rng_int(const Dev& d, Grp& c, int a, int b) { return a + rng_below(d, c, b - a + 1); }

// ---------------------------------------------------------------------------
// World.things queries on the LDS image
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool in_bounds(const Dev& d, int x, int y) { return x >= 0 && y >= 0 && x < d.W && y < d.H; }

__device__ __forceinline__ bool bm_test(const Grp& c, int cell) { return (c.bm[IX(c, cell >> 5)] >> (cell & 31)) & 1u; }
// set / clear as LDS atomics whose result is unused (ds_or_b32 / ds_and_b32): nothing waits on them, and
// a later read of the word by this wave is ordered after them
__device__ __forceinline__ void bm_set(Grp& c, int cell) {
    __hip_atomic_fetch_or(&c.bm[IX(c, cell >> 5)], 1u << (cell & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void bm_clr(Grp& c, int cell) {
    __hip_atomic_fetch_and(&c.bm[IX(c, cell >> 5)], ~(1u << (cell & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// things.get(position) is not None
__device__ __forceinline__ bool occupied(const Dev& d, const Grp& c, int x, int y) {
    return in_bounds(d, x, y) && bm_test(c, y * d.W + x);
}

// things.get(position): entity slot (>= 0), obstacle -(index+1), or NOTHING.  At most one thing stands
// on a cell, so the entity scan has no early exit: its LDS reads issue back to back.
__device__ __forceinline__ int thing_at(const Dev& d, const Grp& c, int x, int y) {
    if (!occupied(d, c, x, y)) return NOTHING;
    const int32_t pk = pack_xy(x, y);
    int hit = -1;
#pragma unroll 4
    for (int s = 0; s < d.E; s++) hit = (LPR(c, s) && LP(c, s) == pk) ? s : hit;
    return hit >= 0 ? hit : -((int)d.cellmap[y * d.W + x] + 1);
}

__device__ __forceinline__ int32_t target_pos(const Dev& d, const Grp& c, int tgt) {
    return tgt >= 0 ? LP(c, tgt) : d.obst_xy[-tgt - 1];
}
__device__ __forceinline__ int target_maxlife(const Dev& d, int tgt) {
    if (tgt >= 0) return 100;  // Zombie / Player / Agent MAX_LIFE (things.py:62,109)
    return d.obst_kind[-tgt - 1] == ZS_THING_BOX ? 10 : 200;
}
__device__ __forceinline__ int target_life(const Dev& d, const Grp& c, int tgt) {
    if (tgt >= 0) return LL(c, tgt);
    return d.obst_hp[(size_t)c.e * d.O + (-tgt - 1)];
}
// v = the new life (64-bit: an obstacle's carried-over life minus a hit may leave the int32 range)
__device__ __forceinline__ void set_target_life(const Dev& d, Grp& c, int tgt, int64_t v) {
    if (tgt >= 0) {  // Zombie / Player / Agent: 100 at most, one tick of hits below 0 at least
        LL(c, tgt) = (int)v;
        return;
    }
    int oi = -tgt - 1;
    d.obst_hp[(size_t)c.e * d.O + oi] = hp_store_value(d, v);
    d.hp_dirty[c.e] |= 1u << (oi / d.hp_chunk);
    uint32_t* w = &d.obst_nonpos[(size_t)c.e * d.OW + (oi >> 5)];
    uint32_t bit = 1u << (oi & 31);
    *w = v <= 0 ? (*w | bit) : (*w & ~bit);
    c.odirty = 1;
}

// closest(...) over present slots [s0, s1) \ {excl}: the first minimum in dict order (branch-free body:
// the slots' LDS reads issue back to back)
__device__ __forceinline__ int closest_in(const Dev& d, const Grp& c, int fx, int fy, int s0, int s1, int excl) {
    if ((d.W - 1) * (d.W - 1) + (d.H - 1) * (d.H - 1) < 65536) {
        // every d^2 of the map fits 16 bits: the minimum of one key (d^2, dict rank, slot) per slot (ranks and
        // slots < 256), the same first minimum in dict order in half the instructions
        const int32_t f = pack_xy(fx, fy);
        uint32_t best = 0xffffffffu;
#pragma unroll 4
        for (int s = s0; s < s1; s++) {
            const uint32_t key = ((uint32_t)d2p(LP(c, s), f) << 16) | ((uint32_t)LR(c, s) << 8) | (uint32_t)s;
            best = (LPR(c, s) && s != excl) ? min(best, key) : best;
        }
        return best == 0xffffffffu ? -1 : (int)(best & 0xffu);
    }
    int best = -1, bd = 0, br = 0;
#pragma unroll 4
    for (int s = s0; s < s1; s++) {
        const bool ok = LPR(c, s) && s != excl;
        const int p = LP(c, s);
        const int dd = d2(fx, fy, unpack_x(p), unpack_y(p));
        const int rk = LR(c, s);
        const bool better = ok && (best < 0 || dd < bd || (dd == bd && rk < br));
        best = better ? s : best;
        bd = better ? dd : bd;
        br = better ? rk : br;
    }
    return best;
}

// ---------------------------------------------------------------------------
// spawning (leader)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void place(const Dev& d, Grp& c, int s, int cell) {
    LP(c, s) = pack_xy(cell % d.W, cell / d.W);
    LPR(c, s) = 1;
    bm_set(c, cell);
    LO(c, c.n_order) = (uint8_t)s;
    c.n_order++;
    d.serial[EIX(d, s, c.e)] = (uint32_t)(++c.serial);
}

// entry i of the player (which = 0) or zombie (which = 1) spawn list, packed x | y << 16
__device__ __forceinline__ int32_t spawn_at(const Dev& d, const Grp& c, int which, int i) {
    if (d.lists_cap) return c.lists[(which ? d.nps : 0) + i];
    return which ? d.zspawn[i] : d.pspawn[i];
}

// World.spawn_in_random (core.py:40-66) for the k slots listed in LM(c, 0..k).  Only the first
// k Fisher-Yates iterations can move the k cells that get popped; the rest are replayed for
// their RNG draws alone.
__device__ __forceinline__ int spawn_in_random(const Dev& d, Grp& c, int k, int which, int nlist, int fail_if_cant) {
    const int total = nlist ? nlist : d.W * d.H;
    const bool lds = total <= d.cand_cap;
    int32_t* gc = d.cand + (size_t)c.e * d.ncand;
#define CGET(i) (lds ? (int)c.cand[IX(c, i)] : gc[i])
#define CSET(i, v)                              \
    do {                                        \
        if (lds) c.cand[IX(c, i)] = (uint16_t)(v); \
        else gc[i] = (v);                       \
    } while (0)
    int n = 0;
    if (nlist == 0) {  // every cell, x-major (core.py:45-47)
        for (int x = 0; x < d.W; x++)
            for (int y = 0; y < d.H; y++) {
                int cell = y * d.W + x;
                if (!bm_test(c, cell)) {
                    CSET(n, cell);
                    n++;
                }
            }
    } else {
        for (int i = 0; i < nlist; i++) {
            int32_t p = spawn_at(d, c, which, i);
            int cell = unpack_y(p) * d.W + unpack_x(p);
            if (!bm_test(c, cell)) {
                CSET(n, cell);
                n++;
            }
        }
    }
    int lim = n - k;
    for (int i = n - 1; i >= 1; i--) {
        int j = rng_below(d, c, i + 1);
        if (i >= lim) {
            int a = CGET(i), b = CGET(j);
            CSET(i, b);
            CSET(j, a);
        }
    }
    for (int m = 0; m < k; m++) {
        int s = LM(c, m);
        if (m < n) {
            place(d, c, s, CGET(n - 1 - m));
        } else {
            if (fail_if_cant) return ZS_ENOSPACE;
            for (int q = m; q < k; q++) LPR(c, LM(c, q)) = 0;  // dropped (game.py:192-194)
            return ZS_OK;
        }
    }
#undef CGET
#undef CSET
    return ZS_OK;
}

// Game.spawn_zombies(count) into free zombie slots (game.py:189-194); every Zombie() draws
// randint(50, 100) before the spawn shuffle (things.py:61-68).
__device__ __forceinline__ void spawn_zombies(const Dev& d, Grp& c, int count) {
    int k = 0;
    for (int s = d.A + d.P; s < d.E && k < count; s++)
        if (!LPR(c, s)) LM(c, k++) = (uint8_t)s;
    for (int i = 0; i < k; i++) {
        int s = LM(c, i);
        LL(c, s) = rng_int(d, c, 50, 100);
        LW(c, s) = ZS_WEAPON_CLAWS;
    }
    spawn_in_random(d, c, k, 1, d.nzs, 0);
}

// a free cell among the zombie spawn candidates (every cell when the map lists none)
__device__ __forceinline__ int any_free_spawn(const Dev& d, const Grp& c) {
    const int total = d.nzs ? d.nzs : d.W * d.H;
    for (int i = 0; i < total; i++) {
        int cell;
        if (d.nzs) {
            int32_t p = spawn_at(d, c, 1, i);
            cell = unpack_y(p) * d.W + unpack_x(p);
        } else {
            cell = i;
        }
        if (!bm_test(c, cell)) return 1;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// decisions on the start-of-tick state.  With rng == false a decision that would draw
// from the RNG returns K_DEFER instead (the leader re-takes it in dict order).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int pick_bit(int mask, int j) {  // j-th set bit (ascending)
    int k = 0;
    for (; k < 4; k++)
        if ((mask >> k) & 1) {
            if (j == 0) break;
            j--;
        }
    return k;
}

// Zombie.next_step (things.py:70-105)
__device__ __forceinline__ void decide_zombie(const Dev& d, Grp& c, int s, bool rng, int& kind, int& tgt) {
    int p = LP(c, s), x = unpack_x(p), y = unpack_y(p);
    int freemask = 0;
    for (int k = 0; k < 4; k++)  // possible_moves: not in things, not bounds-checked (utils.py:47-52)
        if (!occupied(d, c, x + c_adj_dx[k], y + c_adj_dy[k])) freemask |= 1 << k;
    int h = closest_in(d, c, x, y, 0, d.A + d.P, -1);
    if (h >= 0) {
        int hp = LP(c, h), hx = unpack_x(hp), hy = unpack_y(hp);
        if (d2(x, y, hx, hy) <= 2) {  // distance < 1.5
            kind = K_ATTACK;
            tgt = h;
            return;
        }
        if (freemask) {  // closest(target, positions)
            int bk = -1, bd = 0;
            for (int k = 0; k < 4; k++) {
                if (!((freemask >> k) & 1)) continue;
                int dd = d2(hx, hy, x + c_adj_dx[k], y + c_adj_dy[k]);
                if (bk < 0 || dd < bd) {
                    bk = k;
                    bd = dd;
                }
            }
            kind = K_MOVE;
            tgt = pack_xy(x + c_adj_dx[bk], y + c_adj_dy[bk]);
            return;
        }
        // blocked: first Box/Wall in sort_by_distance(target, adjacent_positions(self)).  Every neighbour
        // is occupied (in bounds: an out-of-bounds cell counts as free), so a neighbour no entity stands
        // on holds a present obstacle; one scan of the entities marks the neighbours they stand on.
        int dd[4], em = 0;
        for (int k = 0; k < 4; k++) dd[k] = d2(hx, hy, x + c_adj_dx[k], y + c_adj_dy[k]);
#pragma unroll 4
        for (int t = 0; t < d.E; t++) {
            // the packed offset v = (dx, dy) of thing t: on an adjacent_positions cell when dx^2 + dy^2 == 1;
            // which one from v's bits: (0,1) 0x00010000, (0,-1) 0xffff0000, (1,0) 0x1, (-1,0) 0xffff give
            // (v >> 15 & 3) + (v >> 31) = 2, 3, 0, 1, and ^ 2 the neighbour order 0..3
            const zs_v2s v = __builtin_bit_cast(zs_v2s, LP(c, t)) - __builtin_bit_cast(zs_v2s, p);
            const uint32_t w = __builtin_bit_cast(uint32_t, v);
            const bool on = LPR(c, t) && __builtin_amdgcn_sdot2(v, v, 0, false) == 1;
            em |= on ? 1 << ((((w >> 15) & 3u) + (w >> 31)) ^ 2u) : 0;
        }
        int used = 0;
        for (int r = 0; r < 4; r++) {
            int bk = -1;
            for (int k = 0; k < 4; k++)
                if (!((used >> k) & 1) && (bk < 0 || dd[k] < dd[bk])) bk = k;
            used |= 1 << bk;
            if (!((em >> bk) & 1)) {
                const int bx = x + c_adj_dx[bk], by = y + c_adj_dy[bk];
                kind = K_ATTACK;
                tgt = -((int)d.cellmap[by * d.W + bx] + 1);
                return;
            }
        }
        kind = K_NONE;
        return;
    }
    if (freemask) {  // wander: random.choice(positions)
        if (!rng) {
            kind = K_DEFER;
            return;
        }
        int k = pick_bit(freemask, rng_below(d, c, __popc(freemask)));
        kind = K_MOVE;
        tgt = pack_xy(x + c_adj_dx[k], y + c_adj_dy[k]);
        return;
    }
    kind = K_NONE;
}

__device__ __forceinline__ int clamp16(int v) { return v < -16384 ? -16384 : (v > 16383 ? 16383 : v); }

// Agent.next_step (players/agent.py:28-96) on the action triple
__device__ __forceinline__ void decide_agent(const Dev& d, const Grp& c, int s, int& kind, int& tgt) {
    int p = LP(c, s), x = unpack_x(p), y = unpack_y(p);
    int ak = LACT(c, 3 * s), dx = clamp16(LACT(c, 3 * s + 1)), dy = clamp16(LACT(c, 3 * s + 2));
    kind = K_NONE;
    if (ak == ZS_ACT_MOVE) {
        kind = K_MOVE;
        tgt = pack_xy(x + dx, y + dy);
    } else if (ak == ZS_ACT_ATTACK_CLOSEST) {
        int z = closest_in(d, c, x, y, d.A + d.P, d.E, -1);
        if (z >= 0) {
            kind = K_ATTACK;
            tgt = z;
        }
    } else if (ak == ZS_ACT_ATTACK) {
        int th = thing_at(d, c, x + dx, y + dy);
        if (th != NOTHING) {
            kind = K_ATTACK;
            tgt = th;
        }
    } else if (ak == ZS_ACT_HEAL) {
        if (dx == 0 && dy == 0) {
            kind = K_HEAL;
            tgt = s;
        } else {
            int th = thing_at(d, c, x + dx, y + dy);
            if (th != NOTHING && (th < 0 || th < d.A + d.P)) {  // Player, Box or Wall; never a Zombie
                kind = K_HEAL;
                tgt = th;
            }
        }
    } else if (ak == ZS_ACT_HEAL_CLOSEST) {
        int q = closest_in(d, c, x, y, 0, d.A + d.P, s);
        kind = K_HEAL;
        tgt = q >= 0 ? q : s;
    } else if (ak == ZS_ACT_RAISE && (d.flags & ZS_FLAG_DEBUG)) {
        kind = K_RAISE;  // only a debug env re-raises (core.py:96-99); elsewhere an unknown kind idles
    }
}

// scripted bots (players/{terminator,sniper,troll,hamster,randoman}.py)
__device__ __forceinline__ void decide_bot(const Dev& d, Grp& c, int s, bool rng, int& kind, int& tgt) {
    int p = LP(c, s), x = unpack_x(p), y = unpack_y(p);
    int bt = d.bot_types[s - d.A];
    kind = K_NONE;
    if (bt == ZS_BOT_TERMINATOR) {  // terminator.py:9-37
        int z = closest_in(d, c, x, y, d.A + d.P, d.E, -1);
        if (z < 0) {
            kind = K_HEAL;
            tgt = s;
            return;
        }
        int zp = LP(c, z), zx = unpack_x(zp), zy = unpack_y(zp);
        if (d2(x, y, zx, zy) > weapon_r2(LW(c, s))) {
            int bk = 0, bd = d2(zx, zy, x + c_adj_dx[0], y + c_adj_dy[0]);
            for (int k = 1; k < 4; k++) {
                int dd = d2(zx, zy, x + c_adj_dx[k], y + c_adj_dy[k]);
                if (dd < bd) {
                    bk = k;
                    bd = dd;
                }
            }
            int bx = x + c_adj_dx[bk], by = y + c_adj_dy[bk];
            int th = thing_at(d, c, bx, by);
            if (th != NOTHING) {
                kind = (th >= 0 && th < d.A + d.P) ? K_HEAL : K_ATTACK;
                tgt = th;
            } else {
                kind = K_MOVE;
                tgt = pack_xy(bx, by);
            }
        } else {
            kind = K_ATTACK;
            tgt = z;
        }
    } else if (bt == ZS_BOT_SNIPER) {  // sniper.py:9-19
        int z = closest_in(d, c, x, y, d.A + d.P, d.E, -1);
        if (z >= 0) {
            kind = K_ATTACK;
            tgt = z;
        }
    } else if (bt == ZS_BOT_TROLL) {  // troll.py:10-12
        kind = K_HEAL;
        tgt = s;
    } else if (bt == ZS_BOT_HAMSTER) {  // hamster.py:10-14
        int freemask = 0;
        for (int k = 0; k < 4; k++)
            if (!occupied(d, c, x + c_adj_dx[k], y + c_adj_dy[k])) freemask |= 1 << k;
        if (freemask) {
            if (!rng) {
                kind = K_DEFER;
                return;
            }
            int k = pick_bit(freemask, rng_below(d, c, __popc(freemask)));
            kind = K_MOVE;
            tgt = pack_xy(x + c_adj_dx[k], y + c_adj_dy[k]);
        }
    } else if (bt == ZS_BOT_RANDOMAN) {  // randoman.py:9-21
        if (!rng) {
            kind = K_DEFER;
            return;
        }
        int a = rng_below(d, c, 3);  // choice(('move', 'attack', 'heal'))
        if (a != 0) {
            // choice(list(things.values())): present obstacles (map order), then dynamic things
            const uint32_t* pres = d.obst_present + (size_t)c.e * d.OW;
            int npo = 0;
            for (int w = 0; w < d.OW; w++) npo += __popc(pres[w]);
            int k = rng_below(d, c, npo + c.n_order);
            if (k < npo) {
                int w = 0;
                while (k >= (int)__popc(pres[w])) {
                    k -= __popc(pres[w]);
                    w++;
                }
                uint32_t m = pres[w];
                for (; k > 0; k--) m &= m - 1;
                tgt = -(32 * w + __ffs(m) - 1 + 1);
            } else {
                tgt = LO(c, k - npo);
            }
            kind = a == 1 ? K_ATTACK : K_HEAL;
        } else {
            int axis = rng_below(d, c, 2);            // target[choice((0, 1))]
            int delta = rng_below(d, c, 2) ? 1 : -1;  //   += choice((-1, 1))
            kind = K_MOVE;
            tgt = axis == 0 ? pack_xy(x + delta, y) : pack_xy(x, y + delta);
        }
    }
}

__device__ __forceinline__ void decide(const Dev& d, Grp& c, int s, const int32_t* actions, bool rng, int& kind,
                                       int& tgt) {
    kind = K_NONE;
    tgt = 0;
    if (s < d.A) decide_agent(d, c, s, kind, tgt);
    else if (s < d.A + d.P) decide_bot(d, c, s, rng, kind, tgt);
    else decide_zombie(d, c, s, rng, kind, tgt);
}

// ---------------------------------------------------------------------------
// rules (rules/{extermination,survival,safehouse,evacuation}.py)
// ---------------------------------------------------------------------------
// za0: a zombie is alive beyond the entity table (one a deferred respawn will place)
__device__ __forceinline__ void rules_check(const Dev& d, const Grp& c, int& ended, int& won, int za0 = 0) {
    int pa = 0;  // Rules.players_alive (rules.py:6-11)
    for (int s = 0; s < d.A + d.P; s++) pa |= LL(c, s) > 0;
    if (d.rules == ZS_RULES_EXTERMINATION) {
        int za = za0;
        for (int s = d.A + d.P; s < d.E; s++) za |= LPR(c, s) && LL(c, s) > 0;
        ended = !pa || !za;
        won = pa;
    } else if (d.rules == ZS_RULES_SURVIVAL) {
        ended = !pa;
        won = pa;
    } else if (d.rules == ZS_RULES_SAFEHOUSE) {
        if (pa) {
            int all_in = 1;
            for (int s = 0; s < d.A + d.P; s++) {
                if (LL(c, s) <= 0) continue;
                int p = LP(c, s), cell = unpack_y(p) * d.W + unpack_x(p);
                if (!((d.objbits[cell >> 5] >> (cell & 31)) & 1u)) all_in = 0;
            }
            ended = all_in;
        } else {
            ended = 1;
        }
        won = pa;
    } else {  // evacuation: alive >= half of the team and alive players 4-connected
        int total = d.A + d.P;
        unsigned long long alive = 0;
        int na = 0;
        for (int s = 0; s < total; s++)
            if (LL(c, s) > 0) {
                alive |= 1ull << s;
                na++;
            }
        int half = 2 * na >= total;
        if (half) {
            int first = -1;  // alive_players[0]: first alive bot, else first alive agent
            for (int s = d.A; s < total && first < 0; s++)
                if ((alive >> s) & 1ull) first = s;
            for (int s = 0; s < d.A && first < 0; s++)
                if ((alive >> s) & 1ull) first = s;
            unsigned long long together = 0, frontier = 0;
            if (first >= 0) together = frontier = 1ull << first;
            while (frontier) {
                int s = __ffsll((long long)frontier) - 1;
                frontier &= frontier - 1;
                int p = LP(c, s), x = unpack_x(p), y = unpack_y(p);
                for (int q = 0; q < total; q++) {
                    if (!((alive >> q) & 1ull) || ((together >> q) & 1ull)) continue;
                    int pq = LP(c, q);
                    int dx = unpack_x(pq) - x, dy = unpack_y(pq) - y;
                    if ((dx == 0 && (dy == 1 || dy == -1)) || (dy == 0 && (dx == 1 || dx == -1))) {
                        together |= 1ull << q;
                        frontier |= 1ull << q;
                    }
                }
            }
            ended = __popcll(together) == na;
        } else {
            ended = 1;
        }
        won = half;
    }
}

// ---------------------------------------------------------------------------
// The shuffle and the execution of a tick's actions by the env's G lanes (core.py:76, 103-119).
//
// The reference executes the shuffled actions one at a time, so an action sees every earlier one:
// a move finds its cell taken or freed by earlier moves (core.py:140-166), an attack or heal finds its
// target where an earlier move put it and draws its randint only when in range (core.py:168-202), and
// lives change in order (a heal clamps at MAX_LIFE).  The lanes resolve the same sequence in parallel,
// G actions at a time (a chunk; later chunks see the earlier ones committed):
//   * shuffle: the n - 1 Fisher-Yates draws _randbelow(n - t) are solved over the env's window of
//     tempered MT words with ballots (grp_draws, the fixed point of wave_draws), then lane k follows
//     the element at position k through the swaps;
//   * moves: lane i finds the earlier valid moves that leave or enter its destination cell (one
//     shuffle sweep over the chunk); a move with none of them succeeds iff its cell was free at the
//     chunk's start, the others follow the last earlier successful one of them (freed or taken), in
//     rounds of ballots until every move is resolved (dependencies point to earlier actions only);
//   * attacks / heals: the target's position is the one an earlier successful move of the target gave
//     it, else its chunk-start position; the in-range ones draw their randints in execution order
//     (grp_draws again, one bound per draw), and the last hitter of each target applies every hit on
//     it in order (attack: life - damage; heal: min(MAX_LIFE, life + h));
//   * the chunk's successful moves are committed (occupancy, position, re-insertion at the end of the
//     dict order in execution order: the movers list LM).
// LR (the dict ranks, dead once the decisions are taken) holds the draws; movers are marked 255 in LR
// at the end, as the leader does.  When the window of pre-tempered words cannot hold a chunk's draws,
// the lanes stop before that chunk and the leader takes over (env_step_leader with shuffled = true).
// ---------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ unsigned long long gbits(const Grp& c, unsigned long long b) {
    return G == 64 ? b : (b >> (c.g * G)) & ((1ull << G) - 1ull);
}
template <int G>
__device__ __forceinline__ unsigned long long gballot(const Grp& c, bool p) {
    return gbits<G>(c, __ballot(p));
}

// The window ran out at position pos (every word before it consumed): the G lanes load the stream's next
// rw_step words into it, one round trip, as rng_reload does for the leader.  A block the words cross into
// is twisted first when it is not ready (by lane 0, serially); the refill at the end of every tick and
// reset leaves the next block ready, and a tick draws far fewer than 624 words, so that does not happen
// in practice.
template <int G>
__device__ __forceinline__ void grp_reload(const Dev& d, Grp& c, int& pos) {
    const uint32_t st = st_advance(c.st0, (uint32_t)pos);
    uint32_t off = st & 1023u, slot = (st >> 10) & 1u, ready = (st >> 11) & 1u;
    uint32_t* ring = d.ring + (size_t)c.e * ZS_RING_WORDS;
    const int n = d.rw_step;
    bool twist = false;
    if (off >= ZS_MT_N) {
        twist = !ready;
        if (twist && c.j == 0) mt_twist_serial(ring + (slot ^ 1u) * ZS_MT_N, ring + slot * ZS_MT_N);
        slot ^= 1u;
        off = 0;
        ready = 0;
    }
    if ((int)off + n > ZS_MT_N && !ready) {
        if (c.j == 0) mt_twist_serial(ring + (slot ^ 1u) * ZS_MT_N, ring + slot * ZS_MT_N);
        twist = true;
        ready = 1;
    }
    if (twist) __threadfence();  // lane 0's block before the lanes' loads
    wave_sync();
    for (int k = c.j; k < n; k += G) {
        const uint32_t q = off + k;
        c.rw[IX(c, k)] = mt_temper(q < ZS_MT_N ? ring[slot * ZS_MT_N + q] : ring[(slot ^ 1u) * ZS_MT_N + q - ZS_MT_N]);
    }
    wave_sync();
    c.st0 = st_pack(off, slot, ready);
    c.wlen = n;
    pos = 0;
}

// draws t = 0..count-1 of _randbelow(bound(t)) (random.py:239-249) from the env's window words pos, pos+1, ...
// G words per round: the word of lane j serves draw t_j = done + j - H_j (H_j = rejected words of the round
// before lane j), solved as a fixed point as in wave_draws; a round ends at the window's end, and an empty
// window is reloaded (grp_reload).  put(t, value) for every accepted draw.
template <int G, class Bound, class Put>
__device__ __forceinline__ void grp_draws(const Dev& d, Grp& c, int& pos, int count, Bound bound, Put put) {
    const int j = c.j;
    // the wave's own ballots with per-lane masks of the group (gm) and of its lanes below this one: the fixed
    // point's loop test compares whole-wave masks (scalar), with no per-lane shift of every ballot; a group at
    // its fixed point is unchanged by the iterations the other groups still need
    const unsigned long long gm = G == 64 ? ~0ull : ((1ull << G) - 1ull) << (c.g * G);
    const unsigned long long below = gm & ((1ull << (c.g * G + j)) - 1ull);
    int done = 0;
    while (done < count) {
        if (pos >= c.wlen) grp_reload<G>(d, c, pos);
        const bool avail = pos + j < c.wlen;
        const uint32_t w = avail ? c.rw[IX(c, pos + j)] : 0u;
        unsigned long long rej = 0ull, prev;
        int t, b;
        bool lv, rj;
        do {
            prev = rej;
            t = done + j - __popcll(rej & below);
            lv = avail && t < count;
            b = lv ? bound(t) : 1;
            rj = lv && (w >> (__clz(b))) >= (uint32_t)b;  // getrandbits(bit_length(b)) = w >> (32 - bit_length(b))
            rej = __ballot(rj);
        } while (rej != prev);
        const unsigned long long live = __ballot(lv) & gm;
        if (lv && !rj) put(t, w >> __clz(b));
        done += __popcll(live) - __popcll(rej & gm);
        pos += 64 - __clzll((long long)live) - c.g * G;
    }
}

// random.shuffle of the n actions LPE(0..n) (n <= 2G) from window word pos on.  The draws go to the
// env's first table as bytes (4G of them).
template <int G>
__device__ __forceinline__ void grp_shuffle(const Dev& d, Grp& c, int n, int& pos) {
    if (n < 2) return;
    GX_DECL
    GX(0);
    lu8* jt8 = (lu8*)(c.xs + c.g * G);
    grp_draws<G>(d, c, pos, n - 1, [&](int t) { return n - t; }, [&](int t, uint32_t v) { jt8[t] = (uint8_t)v; });
    wave_sync();
    GX(1);
    // the swaps (i = n - 1 - t with j_t), in order, by the env's leader lane on the LDS list.  The tick is
    // VALU-bound where it matters (C3-C5: every instruction issues for the whole wave), and this chain is
    // ~5 instructions a swap against ~16 for every lane following two elements through all the swaps (C5:
    // the shuffle 803 VALU instructions per wave of 4 envs, profiles/r06v_pmc_stop.log); its LDS round trips
    // run under the other waves' issue.
    if (c.j == 0) {
        const lu32* jw = (const lu32*)jt8;
        for (int t0 = 0; t0 < n - 1; t0 += 4) {
            const uint32_t q = jw[t0 >> 2];
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int t = t0 + b;
                if (t < n - 1) {
                    const int i = n - 1 - t, jt = (int)((q >> (8 * b)) & 0xffu);
                    const uint8_t x = LPE(c, i), y = LPE(c, jt);
                    LPE(c, i) = y;
                    LPE(c, jt) = x;
                }
            }
        }
    }
    wave_sync();
    GX(2);
}

// execute the shuffled actions LPE(0..n) chunk by chunk.  Successful movers are appended to LM(nmoved..);
// odirty is set when an obstacle was hit.  The lanes
// exchange their actions through the env's two tables (t0, t1: one word per lane), read back four
// words at a time.
#ifndef ZS_DIAG_STOP
#define ZS_DIAG_STOP 0  // diagnostic builds only (tick_wg): 7-10 end each chunk of grp_execute early
#endif
template <int G>
__device__ __forceinline__ void grp_execute(const Dev& d, Grp& c, int n, int& pos, int& nmoved, int& odirty) {
    const int j = c.j;
    const unsigned long long below = (1ull << j) - 1ull;
    const unsigned long long gfull = G == 64 ? ~0ull : (1ull << G) - 1ull;
    li32* t0 = c.xs + c.g * G;
    li32* t1 = c.xs + 64 + c.g * G;
    const ZS_LDS zs_v4i* t0v = (const ZS_LDS zs_v4i*)t0;
    const ZS_LDS zs_v4i* t1v = (const ZS_LDS zs_v4i*)t1;
    GX_DECL
    GX(0);
    for (int c0 = 0; c0 < n; c0 += G) {
        const int m = min(G, n - c0);
        const bool act = j < m;
        // the scans below stop at the wave's longest chunk (entries past an env's m hold no move / no hit),
        // rounded up to the 4-entry reads
        int mw;
        {
            const unsigned long long am = __ballot(act);
            unsigned long long comb = 0ull;
#pragma unroll
            for (int g = 0; g < 64 / G; g++) comb |= (am >> (g * G)) & gfull;
            mw = min(G, (64 - __clzll((long long)comb) + 3) & ~3);
        }
        int s = 0, kind = K_NONE, tgt = 0, p = 0, w = 0;
        if (act) {
            s = LPE(c, c0 + j);
            kind = LK(c, s);
            tgt = LT(c, s);
            p = LP(c, s);
            w = LW(c, s);
        }
        const int px = unpack_x(p), py = unpack_y(p);
        // a valid move: in bounds and one step (core.py:140-166); it still fails on an occupied cell
        bool mv = false;
        int dcell = 0;
        if (kind == K_MOVE) {
            const int tx = unpack_x(tgt), ty = unpack_y(tgt);
            mv = in_bounds(d, tx, ty) && d2(px, py, tx, ty) <= 1;
            dcell = ty * d.W + tx;
        }
        t0[j] = mv ? tgt : -1;  // valid moves' destinations (packed, >= 0) and sources (-2: not a valid move)
        t1[j] = mv ? p : -2;
        if (act) LR(c, s) = (uint8_t)j;  // the chunk position of each actor (dict ranks are dead by now)
        const bool occ0 = mv && bm_test(c, dcell);
        const bool hits = kind == K_ATTACK || kind == K_HEAL;
        const int et = hits && tgt >= 0 ? tgt : -1;  // an entity target may have moved earlier
        // an obstacle target's position, kind and life: one round of global loads
        int tp0 = 0, okind = 0, ohp = 0;
        if (hits && tgt < 0) {
            tp0 = d.obst_xy[-tgt - 1];
            okind = d.obst_kind[-tgt - 1];
            ohp = d.obst_hp[(size_t)c.e * d.O + (-tgt - 1)];
        } else if (et >= 0) {
            tp0 = LP(c, et);
        }
        wave_sync();
        GX(3);
        if (ZS_DIAG_STOP == 7) continue;
        // earlier valid moves of the chunk that leave (vac) or enter (dep) this move's cell.  A lane without a
        // valid move wrote no cell (-1 / -2 match no destination), so the scan compares cells alone, four
        // entries to a nibble, and the earlier-lanes and valid-move conditions apply once, to the masks
        typedef typename std::conditional<G <= 32, uint32_t, unsigned long long>::type MaskT;
        MaskT depm = 0, vacm = 0;
        constexpr int UNR = G <= 16 ? G / 4 : 2;  // whole scans up to 16 lanes; wider groups by halves of 8
#pragma unroll UNR
        for (int k0 = 0; k0 < mw; k0 += 4) {
            const zs_v4i dv = t0v[k0 >> 2], sv = t1v[k0 >> 2];
            uint32_t vn = 0u, dn = 0u;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const bool a = sv[u] == tgt;
                vn |= a ? 1u << u : 0u;
                dn |= (a || dv[u] == tgt) ? 1u << u : 0u;
            }
            vacm |= (MaskT)vn << k0;
            depm |= (MaskT)dn << k0;
        }
        const MaskT ltm = (MaskT)((1ull << j) - 1ull);
        const unsigned long long vac = mv ? (unsigned long long)(vacm & ltm) : 0ull;
        const unsigned long long dep = mv ? (unsigned long long)(depm & ltm) : 0ull;
        // the target's own move earlier in the chunk
        int tmv = -1, tdst = 0;
        if (et >= 0) {
            const int k = LR(c, et);
            if (k < j && LPE(c, c0 + k) == et) {
                tdst = t0[k];
                tmv = tdst >= 0 ? k : -1;
            }
        }
        GX(4);
        if (ZS_DIAG_STOP == 8) continue;
        bool res = !mv || dep == 0ull;
        bool suc = mv && dep == 0ull && !occ0;
        unsigned long long R = gballot<G>(c, res), S = gballot<G>(c, suc);
        while (R != gfull) {
            if (!res && (dep & ~R) == 0ull) {
                const unsigned long long sd = dep & S;
                suc = sd ? ((vac >> (63 - __clzll((long long)sd))) & 1ull) != 0ull : !occ0;
                res = true;
            }
            R = gballot<G>(c, res);
            S = gballot<G>(c, suc);
        }
        // attacks / heals: in range at the target's position of the moment (core.py:168-202)
        bool inr = false;
        int lo = 0, bnd = 1, ml = 100;
        if (hits) {
            ml = tgt >= 0 ? 100 : okind == ZS_THING_BOX ? 10 : 200;  // target_maxlife
            const int tp = (tmv >= 0 && ((S >> tmv) & 1ull)) ? tdst : tp0;
            if (kind == K_ATTACK) {
                inr = d2(px, py, unpack_x(tp), unpack_y(tp)) <= weapon_r2(w);
                lo = weapon_lo(w);
                bnd = weapon_hi(w) - lo + 1;
            } else {
                inr = d2(px, py, unpack_x(tp), unpack_y(tp)) <= 9;
                lo = ml / 10;
                bnd = ml / 4 - lo + 1;
            }
        }
        GX(5);
        if (ZS_DIAG_STOP == 9) continue;
        const unsigned long long IR = gballot<G>(c, inr);
        const int r = __popcll(IR & below);
        wave_sync();  // the scans' table reads before the bounds overwrite t1
        if (inr) t1[r] = bnd;
        wave_sync();
        grp_draws<G>(d, c, pos, __popcll(IR), [&](int t) { return (int)t1[t]; }, [&](int t, uint32_t v) { t1[t] = (int)v; });
        wave_sync();
        GX(6);
        if (ZS_DIAG_STOP == 10) continue;
        // every hit on a target in execution order; the last hitter stores the result
        const int hv = inr ? (kind == K_ATTACK ? -(lo + t1[r]) : lo + t1[r]) : 0;
        wave_sync();
        t0[j] = inr ? tgt : 0x7fffffff;  // hit targets (0x7fffffff: no hit) and signed hit values
        t1[j] = hv;
        wave_sync();
        int life = 0;
        if (inr) life = tgt >= 0 ? LL(c, tgt) : ohp;
        bool last = inr;
        uint32_t ovf = 0u;  // an obstacle's life after one of the hits left the int16 / int32 range
        const bool ohit = __ballot(inr && tgt < 0) != 0ull;  // some obstacle is hit in the wave's chunks
        if (!ohit && __ballot(inr && life > 100) == 0ull) {
            // entity targets at most at MAX_LIFE (the common chunk; only a state poke sets more): no hit
            // saturates, and min(life + hit, 100) is both an attack (hit < 0) and a capped heal.  A lane that
            // hits nothing ends with last = false and an unused life, so the entries need no inr test; a
            // no-hit entry's target (0x7fffffff) matches no lane's.  The same values as the loop below.
#pragma unroll UNR
            for (int k0 = 0; k0 < mw; k0 += 4) {
                const zs_v4i tv = t0v[k0 >> 2], hvv = t1v[k0 >> 2];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int k = k0 + u;
                    const bool same = tv[u] == tgt;
                    const int nl = min(life + hvv[u], 100);
                    life = (same && k <= j) ? nl : life;
                    last = last && !(same && k > j);
                }
            }
        } else {
#pragma unroll UNR
        for (int k0 = 0; k0 < mw; k0 += 4) {
            const zs_v4i tv = t0v[k0 >> 2], hvv = t1v[k0 >> 2];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int k = k0 + u;
                const bool app = inr && tv[u] == tgt && k <= j;
                const int hk = hvv[u];
                // a hit is at most 100: life + hk leaves int32 only below ZS_HP_FLOOR, where an obstacle's life
                // saturates (hp_store_value of every hit, as the leader stores them); a heal clamps at MAX_LIFE
                const bool sat = hk < 0 && life < ZS_HP_FLOOR - hk;
                const int nl = sat ? ZS_HP_FLOOR : (hk < 0 ? life + hk : min(life + hk, ml));
                if (tgt < 0) {
                    ovf |= (app && nl < -32768) ? ZS_OVF_INT16 : 0u;
                    ovf |= (app && sat) ? ZS_OVF_INT32 : 0u;
                }
                life = app ? nl : life;
                last = last && !(inr && tv[u] == tgt && k > j);
            }
        }
        }
        if (last) {
            if (tgt >= 0) {
                LL(c, tgt) = (int)life;
            } else {  // set_target_life's obstacle path, one lane per obstacle
                const int oi = -tgt - 1;
                if (ovf && (__hip_atomic_load(d.ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ovf) != ovf)
                    atomicOr(d.ovf, ovf);
                d.obst_hp[(size_t)c.e * d.O + oi] = (int32_t)life;
                atomicOr(&d.hp_dirty[c.e], 1u << (oi / d.hp_chunk));
                uint32_t* wp = &d.obst_nonpos[(size_t)c.e * d.OW + (oi >> 5)];
                if (life <= 0) atomicOr(wp, 1u << (oi & 31));
                else atomicAnd(wp, ~(1u << (oi & 31)));
            }
        }
        if (ohit && gballot<G>(c, inr && tgt < 0)) odirty = 1;
        // commit the chunk's moves: cells freed before cells taken (a cell is left at most once and
        // taken at most once per tick, in that order), positions, movers in execution order
        if (suc) bm_clr(c, py * d.W + px);
        if (suc) {
            bm_set(c, dcell);
            LP(c, s) = tgt;
            LM(c, nmoved + __popcll(S & below)) = (uint8_t)s;
        }
        nmoved += __popcll(S);
        wave_sync();
        GX(7);
    }
}

// ---------------------------------------------------------------------------
// leader: the order-dependent rest of the tick (gym_env.py:99-145 / multiagent_env.py:111-171), where the
// env's lanes did not execute the actions (a decision deferred to the leader, or more than 2G actions)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void env_step_leader(const Dev& d, Grp& c, const int32_t* actions, double* rew, uint8_t* done_out,
                                uint8_t* trunc_out, uint8_t* listed_out) {
    const int A = d.A;
    SUB_DECL
    SUB(0);
    // World.get_actions (core.py:80-101): deferred (RNG-drawing) decisions in dict order (the action
    // list is already compacted when there are none)
    int nact = MISC(c, MISC_NMOVED);
    const bool serial = nact < 0;
    if (serial) nact = 0;
    for (int k = 0; k < c.n_order && serial; k++) {
        int s = LO(c, k);
        if (LK(c, s) == K_RAISE) {
            // this agent's next_step raised and the env re-raises (debug, core.py:96-99): the step
            // stops here, after t += 1 and the earlier actors' decisions (and their draws)
            const int nr = d.reward_mode == ZS_REWARD_SINGLE ? 1 : A;
            for (int a = 0; a < nr; a++) rew[(size_t)c.e * nr + a] = 0.0;
            if (listed_out)
                for (int a = 0; a < A; a++) listed_out[(size_t)c.e * A + a] = (uint8_t)MISC(c, MISC_N + A + a);
            done_out[c.e] = 0;
            trunc_out[c.e] = 0;
            c.fin = 0;
            c.respawn = 0;
            MISC(c, MISC_NMOVED) = -1;  // no cleanup, no second leader part
            if (d.alog) {  // the actors before it that decided an action, in dict order; -1 - their count
                int32_t* al = d.alog + (size_t)c.e * d.E * 2;
                for (int j = 0; j < nact; j++) {
                    const int sj = LPE(c, j);
                    al[2 * j] = sj | (LK(c, sj) << 8);
                    al[2 * j + 1] = LT(c, sj);
                }
                d.alog_n[c.e] = -1 - nact;
            }
            return;
        }
        if (LK(c, s) == K_DEFER) {
            int kind, tgt;
            decide(d, c, s, actions, true, kind, tgt);
            LK(c, s) = (uint8_t)kind;
            LT(c, s) = tgt;
        }
        if (LK(c, s) != K_NONE) LPE(c, nact++) = (uint8_t)s;
    }
    // random.shuffle(actions) (core.py:76)
    for (int i = nact - 1; i >= 1; i--) {
        int j = rng_below(d, c, i + 1);
        uint8_t tmp = LPE(c, i);
        LPE(c, i) = LPE(c, j);
        LPE(c, j) = tmp;
    }
    SUB(1);
    if (d.alog) {  // the executed actions in execution order (drop-in views)
        int32_t* al = d.alog + (size_t)c.e * d.E * 2;
        for (int k = 0; k < nact; k++) {
            const int s = LPE(c, k);
            al[2 * k] = s | (LK(c, s) << 8);
            al[2 * k + 1] = LT(c, s);
        }
        d.alog_n[c.e] = nact;
    }
    // execute_actions (core.py:103-119).  The next action's actor, kind, target and position are read
    // ahead: nothing this action does changes them (every actor acts once, and only its own action moves it).
    int nmoved = 0;
    int s_n = 0, kind_n = K_NONE, tgt_n = 0, p_n = 0;
    if (nact > 0) {
        s_n = LPE(c, 0);
        kind_n = LK(c, s_n);
        tgt_n = LT(c, s_n);
        p_n = LP(c, s_n);
    }
    for (int i = 0; i < nact; i++) {
        const int s = s_n, kind = kind_n, tgt = tgt_n, p = p_n, x = unpack_x(p), y = unpack_y(p);
        if (i + 1 < nact) {
            s_n = LPE(c, i + 1);
            kind_n = LK(c, s_n);
            tgt_n = LT(c, s_n);
            p_n = LP(c, s_n);
        }
        if (kind == K_MOVE) {  // thing_move (core.py:140-166)
            int tx = unpack_x(tgt), ty = unpack_y(tgt);
            if (in_bounds(d, tx, ty) && !bm_test(c, ty * d.W + tx) && d2(x, y, tx, ty) <= 1) {
                bm_clr(c, y * d.W + x);
                bm_set(c, ty * d.W + tx);
                LP(c, s) = tgt;
                LM(c, nmoved++) = (uint8_t)s;
                LR(c, s) = 255;  // re-inserted at the end of the dict
            }
        } else if (kind == K_ATTACK) {  // thing_attack (core.py:168-184)
            int tp = target_pos(d, c, tgt);
            int w = LW(c, s);
            if (d2(x, y, unpack_x(tp), unpack_y(tp)) <= weapon_r2(w)) {
                int dmg = rng_int(d, c, weapon_lo(w), weapon_hi(w));
                set_target_life(d, c, tgt, (int64_t)target_life(d, c, tgt) - dmg);
            }
        } else {  // thing_heal (core.py:186-202), HEALING_RANGE = 3
            int tp = target_pos(d, c, tgt);
            if (d2(x, y, unpack_x(tp), unpack_y(tp)) <= 9) {
                int ml = target_maxlife(d, tgt);
                int hl = rng_int(d, c, ml / 10, ml / 4);
                const int64_t nl = (int64_t)target_life(d, c, tgt) + hl;
                set_target_life(d, c, tgt, nl < ml ? nl : (int64_t)ml);
            }
        }
    }
    SUB(2);
    // the group's lanes rebuild the dict order and clean up the dead (env_cleanup_group)
    MISC(c, MISC_NMOVED) = nmoved;
    MISC(c, MISC_NORD) = c.n_order;
    MISC(c, MISC_DEATHS) = c.deaths;
    MISC(c, MISC_ZD) = c.zd;
    MISC(c, MISC_ODIRTY) = c.odirty;
}

// clean_dead_things (core.py:121-138) and the dict order after the tick's moves (unmoved things in the
// old order, then the movers in execution order, core.py:158-159), by the G lanes of the env: every
// entry is a lane of a chunk, the survivors are compacted with a ballot, the dead ones leave a DeadBody
// (any order: two things never share a cell) and are counted with LDS atomics.  The obstacles that
// dropped to life <= 0 go the same way (one word of present bits per lane).
template <int G>
__device__ __forceinline__ void env_cleanup_group(const Dev& d, Grp& c, bool run) {
    const int A = d.A, j = c.j;
    const bool stepping_ = run;
    const int nm = run ? MISC(c, MISC_NMOVED) : -1;
    run = run && nm >= 0;  // nm < 0: this step re-raised an agent's exception (debug) and ended there
    const int K = run ? MISC(c, MISC_NORD) : 0;
    if (run && MISC(c, MISC_ODIRTY)) {
        for (int w = j; w < d.OW; w += G) {
            uint32_t* pw = &d.obst_present[(size_t)c.e * d.OW + w];
            const uint32_t pv = *pw;
            uint32_t dead = pv & d.obst_nonpos[(size_t)c.e * d.OW + w];
            if (dead) {
                *pw = pv & ~dead;
                __hip_atomic_fetch_add(&MISC(c, MISC_DEATHS), (int)__popc(dead), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                while (dead) {
                    const int32_t op = d.obst_xy[32 * w + __ffs(dead) - 1];
                    dead &= dead - 1;
                    const int cell = unpack_y(op) * d.W + unpack_x(op);
                    __hip_atomic_fetch_and(&c.bm[IX(c, cell >> 5)], ~(1u << (cell & 31)), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
    }
    const int total = run ? K + nm : 0;
    uint32_t* deadbits = d.dead + (size_t)c.e * d.DW;
    int kept = 0, nlog = 0;
    for (int b0 = 0; b0 < total; b0 += G) {
        const int idx = b0 + j;
        int s = 0;
        bool keep = false;
        if (idx < total) {
            s = idx < K ? LO(c, idx) : LM(c, idx - K);
            const bool incl = idx >= K || LR(c, s) != 255;
            keep = incl && LL(c, s) > 0;
            if (incl && !keep) {
                const int32_t p = LP(c, s);
                const int cell = unpack_y(p) * d.W + unpack_x(p);
                __hip_atomic_fetch_or(&deadbits[cell >> 5], 1u << (cell & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);  // DeadBody decoration
                __hip_atomic_fetch_or(&d.dead_dirty[c.e], 1u << ((cell >> 5) / d.dead_chunk), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_and(&c.bm[IX(c, cell >> 5)], ~(1u << (cell & 31)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                LPR(c, s) = 0;
                __hip_atomic_fetch_add(&MISC(c, MISC_DEATHS), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (s >= A + d.P)
                    __hip_atomic_fetch_add(&MISC(c, MISC_ZD), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        const unsigned long long bal = __ballot(keep);
        const unsigned long long gb = G == 64 ? bal : (bal >> (c.g * G)) & ((1ull << G) - 1ull);
        if (keep) LO(c, kept + __popcll(gb & ((1ull << j) - 1ull))) = (uint8_t)s;
        kept += __popcll(gb);
        if (d.dlog) {  // ZS_FLAG_DEATH_LOG: the removed things in dict order
            const bool gone = idx < total && (idx >= K || LR(c, s) != 255) && !keep;
            const unsigned long long db = __ballot(gone);
            const unsigned long long gd = G == 64 ? db : (db >> (c.g * G)) & ((1ull << G) - 1ull);
            if (gone) {
                int32_t* en = d.dlog + ((size_t)c.e * d.E + nlog + __popcll(gd & ((1ull << j) - 1ull))) * 5;
                const int32_t p = LP(c, s);
                en[0] = s;
                en[1] = (int32_t)d.serial[EIX(d, s, c.e)];
                en[2] = unpack_x(p);
                en[3] = unpack_y(p);
                en[4] = LL(c, s);
            }
            nlog += __popcll(gd);
        }
    }
    if (d.dlog && stepping_ && j == 0) d.dlog_n[c.e] = nlog;
    // what the leader's respawn and rules read, from the cleaned-up table: present zombies, any player
    // alive (Rules.players_alive), any agent alive, an alive player off the objectives (Safehouse)
    int nz = 0;
    unsigned long long pa = 0ull, aa = 0ull, off = 0ull;
    const unsigned long long gmask = G == 64 ? ~0ull : ((1ull << G) - 1ull) << (c.g * G);
    for (int s0 = 0; s0 < (run ? d.E : 0); s0 += G) {
        const int s = s0 + j;
        bool z = false, al = false, ag = false, o = false;
        if (s < d.E) {
            if (s >= A + d.P) {
                z = LPR(c, s) != 0;
            } else {
                al = LL(c, s) > 0;
                ag = al && s < A;
                if (al && d.rules == ZS_RULES_SAFEHOUSE) {
                    const int32_t p = LP(c, s);
                    const int cell = unpack_y(p) * d.W + unpack_x(p);
                    o = !((d.objbits[cell >> 5] >> (cell & 31)) & 1u);
                }
            }
        }
        nz += __popcll(__ballot(z) & gmask);
        pa |= __ballot(al) & gmask;
        aa |= __ballot(ag) & gmask;
        off |= __ballot(o) & gmask;
    }
    if (run && j == 0) {
        MISC(c, MISC_NORD) = kept;
        MISC(c, MISC_NMOVED) = nz | (pa ? 1 << 16 : 0) | (aa ? 1 << 17 : 0) | (off ? 1 << 18 : 0);
    }
}

// the rest of the tick after the group's cleanup (leader)
__device__ __forceinline__ void env_step_leader_b(const Dev& d, Grp& c, double* rew, uint8_t* done_out, uint8_t* trunc_out,
                                                  uint8_t* listed_out) {
    const int A = d.A;
    SUB_DECL
    SUB(0);
    c.n_order = MISC(c, MISC_NORD);
    c.deaths = MISC(c, MISC_DEATHS);
    c.zd = MISC(c, MISC_ZD);
    c.odirty = 0;
    const int gfl = MISC(c, MISC_NMOVED);
    const int nz = gfl & 0xffff, pa = (gfl >> 16) & 1, aa = (gfl >> 17) & 1, off = (gfl >> 18) & 1;
    SUB(3);
    // reward_tracker.update (gym/reward.py:30-35, 77-86)
    double rs = 0.0;
    if (d.reward_mode == ZS_REWARD_SINGLE) {
        long long sp = 0, sc = 0;
        for (int a = 0; a < A; a++) {
            sp += MISC(c, MISC_N + a);
            sc += LL(c, a);
        }
        double prev = (double)c.prevzd + (double)sp / 100.0;
        double cur = (double)c.zd + (double)sc / 100.0;
        rs = cur - prev;
    }
    // the multi-agent deltas are formed where they are written, after the rules (respawn and rules
    // change no agent's life and no death count): reading back a stored delta would wait for every
    // store the wave has in flight
    // spawn_zombies_to_maintain_minimum (game.py:196-201).  Deferred: the respawn is the step's
    // last RNG consumer and nothing below reads the new zombies except Extermination's "any zombie
    // alive", which only needs to know whether one more zombie gets placed (a free spawn cell).
    int za0 = 0, spawned = 0;
    c.respawn = 0;
    if (nz < d.minimum_zombies) {
        if (d.defer_respawn) {
            c.respawn = 1;
            if (nz == 0 && d.rules == ZS_RULES_EXTERMINATION) za0 = any_free_spawn(d, c);
        } else {
            spawn_zombies(d, c, d.minimum_zombies - nz);
            spawned = 1;
        }
    }
    // rules and end-of-game reward (gym_env.py:130-141, gym/multiagent_env.py:143-162); the group's
    // counts stand unless this step placed zombies (Extermination then looks again)
    int ended, won, tr = 0;
    if (d.rules == ZS_RULES_EVACUATION || (spawned && d.rules == ZS_RULES_EXTERMINATION)) {
        rules_check(d, c, ended, won, za0);
    } else {
        won = pa;
        ended = d.rules == ZS_RULES_EXTERMINATION ? (!pa || !(nz > 0 || za0))
                : d.rules == ZS_RULES_SAFEHOUSE   ? (!pa || !off)
                                                  : !pa;
    }
    double end_reward = 0.0;
    if (ended) {
        end_reward = won ? 10.0 : -10.0;
    } else {
        if (!aa) {
            tr = 1;
            end_reward = -10.0;
        }
    }
    if (d.reward_mode == ZS_REWARD_SINGLE) {
        if (ended || tr) rs += end_reward;
        rew[c.e] = rs;
        if (listed_out)
            for (int a = 0; a < A; a++) listed_out[(size_t)c.e * A + a] = (uint8_t)MISC(c, MISC_N + A + a);
    } else {
        // the per-agent deltas are formed by the agents' lanes after the leader's part (multi_rewards): the
        // leader leaves the end reward and the reward tracker's old zombie-death count in the scratch rows
        MISC(c, MISC_NMOVED) = ended ? (won ? 1 : 2) : (end_reward != 0.0 ? 2 : 0);
        MISC(c, MISC_NORD) = c.prevzd;
    }
    if (d.reward_mode == ZS_REWARD_SINGLE)
        for (int a = 0; a < A; a++) MISC(c, MISC_N + a) = LL(c, a);
    c.prevzd = c.zd;
    c.epsteps++;
    if (d.max_steps > 0 && c.epsteps >= d.max_steps) tr = 1;
    done_out[c.e] = (uint8_t)ended;
    trunc_out[c.e] = (uint8_t)tr;
    c.fin = ended || tr;
    SUB(4);
}

// MultiAgentRewards.update and the end-of-game rewards (gym/reward.py:77-98, gym/multiagent_env.py:143-162)
// for the agents of a stepping env, one agent per lane of the env's group (agent a on lane a mod G), after
// env_step_leader_b left the end reward (MISC_NMOVED: 0 none, 1 +10, 2 -10) and the tracker's previous
// zombie-death count (MISC_NORD); the same float64 operations in the same order as the reference.  Also
// env.agents for the next step (alive after this one) and the tracker's lives.
__device__ __forceinline__ void multi_rewards(const Dev& d, const Grp& c, double* rew, uint8_t* listed_out) {
    const int A = d.A, code = MISC(c, MISC_NMOVED), prevzd = MISC(c, MISC_NORD), zd = MISC(c, MISC_ZD);
    const double end_reward = code == 1 ? 10.0 : (code == 2 ? -10.0 : 0.0);
    for (int a = c.j; a < A; a += 64 / c.ne) {  // G = 64 / ne lanes per env
        const uint8_t was = (uint8_t)MISC(c, MISC_N + A + a);
        const int life = LL(c, a);
        if (listed_out) listed_out[(size_t)c.e * A + a] = was;
        const double prev = (double)prevzd + (double)MISC(c, MISC_N + a) / 100.0;
        const double cur = (double)zd + (double)life / 100.0;
        double r = cur - prev;
        if (!was) r = 0.0;
        else if (life > 0) r = r + end_reward;
        rew[(size_t)c.e * A + a] = r;
        MISC(c, MISC_N + A + a) = life > 0;
        MISC(c, MISC_N + a) = life;
    }
}

// ---------------------------------------------------------------------------
// wave-cooperative MT19937 refill: every env of the workgroup whose next block is not ready gets it
// twisted by all 64 lanes (3 dependency phases over the 624-word block): one round of 10 loads per
// lane, the phases in LDS, the stores.  No workgroup barrier: nothing this wave stored earlier is read
// (a serial twist of the tick is followed by its own fence), so the loads do not wait for its stores.
// ---------------------------------------------------------------------------
// env e's next block (slot ^ 1 of the stream state st) twisted by one wave through tw (2 x 624 LDS
// words of that wave), then marked ready in the env's stream state
__device__ __forceinline__ void wave_refill(const Dev& d, int e, uint32_t st, lu32* tw, int lane) {
    constexpr int K = (ZS_MT_N + 63) / 64;
    const uint32_t slot = (st >> 10) & 1u;
    uint32_t* ring = d.ring + (size_t)e * ZS_RING_WORDS;
    const uint32_t* src = ring + slot * ZS_MT_N;
    uint32_t* dst = ring + (slot ^ 1u) * ZS_MT_N;
    uint32_t v[K];
#pragma unroll
    for (int u = 0; u < K; u++) v[u] = src[min(lane + 64 * u, ZS_MT_N - 1)];
    wave_sync();
#pragma unroll
    for (int u = 0; u < K; u++)
        if (lane + 64 * u < ZS_MT_N) tw[lane + 64 * u] = v[u];
    wave_sync();
    lu32* nw = tw + ZS_MT_N;
    lds_twist(tw, nw, lane);
    wave_sync();
    for (int k = lane; k < ZS_MT_N; k += 64) dst[k] = nw[k];
    if (lane == 0) d.rngst[e] = st | (1u << 11);
    wave_sync();
}

__device__ __forceinline__ void coop_refill(const Dev& d, int base, int count, const lu32* lst, lu32* tw) {
    for (int i = 0; i < count; i++) {
        const uint32_t st = lst[i];
        if (!((st >> 11) & 1u)) wave_refill(d, base + i, st, tw, threadIdx.x & 63);
    }
}


// The HBM home of MISC row f of env e (MISC_NMOVED / MISC_NORD: none): an int32 word of the scalar rows
// or of prev_life, or (listed, rows MISC_N + A ..) a byte, as one address select instead of a branch per
// row (every row a separate masked load or store)
static_assert(MISC_T == S_T && MISC_DEATHS == S_DEATHS && MISC_ZD == S_ZD && MISC_EPSTEPS == S_EPSTEPS &&
                  MISC_PREVZD + 2 == S_PREVZD && MISC_SERIAL + 2 == S_SERIAL && MISC_ODIRTY + 2 == S_ODIRTY,
              "MISC rows -> scalar rows");
__device__ __forceinline__ int32_t* misc_word(const Dev& d, int f, int e) {
    const size_t N = d.N;
    return f < MISC_NMOVED ? d.scal + (size_t)(f < MISC_PREVZD ? f : f + 2) * N + e
                           : d.prev_life + (size_t)(f - MISC_N) * N + e;  // f < MISC_N + A
}
__device__ __forceinline__ int misc_load(const Dev& d, int f, int e) {
    if (f >= MISC_N + d.A) return d.listed[(size_t)(f - MISC_N - d.A) * d.N + e];
    const int v = *misc_word(d, f < MISC_NMOVED || f >= MISC_N ? f : 0, e);
    return f == MISC_NMOVED || f == MISC_NORD ? 0 : v;
}
__device__ __forceinline__ void misc_store(const Dev& d, int f, int e, int v) {
    if (f == MISC_NMOVED || f == MISC_NORD) return;
    if (f >= MISC_N + d.A) d.listed[(size_t)(f - MISC_N - d.A) * d.N + e] = (uint8_t)v;
    else *misc_word(d, f, e) = v;
}

// word v into every env's copy of LDS row w (IX layout: row w of env g at w * NE + g), one store
template <int NE>
__device__ __forceinline__ void bcast_row(lu32* base, int w, uint32_t v) {
    if constexpr (NE == 1) {
        base[w] = v;
    } else if constexpr (NE == 2) {
        *(ZS_LDS zs_v2u*)(base + 2 * w) = zs_v2u{v, v};
    } else {
#pragma unroll
        for (int k = 0; k < NE / 4; k++) *(lv4u*)(base + w * NE + 4 * k) = zs_v4u{v, v, v, v};
    }
}

// ---------------------------------------------------------------------------
// k_tick: one workgroup = one wave = 64/G envs
// ---------------------------------------------------------------------------
// envs [env0, env1) of this launch; workgroup wg takes the NE envs from env0 + wg * NE.
// EARLY (the one-round fused launch, whose register budget has room): the RNG window's first 4G words
// are loaded in registers right after the first load round and reach LDS only after the decisions, so
// their round trip (it needs the stream state) overlaps the decisions instead of the stage-in
// smem: this wave's LDS image (tick_layout)
#ifndef ZS_TICK_LAUNDER
#define ZS_TICK_LAUNDER 1
#endif

template <int G, bool EARLY = false>
__device__ __forceinline__ void tick_wg(const Dev& d0, int wg, const int32_t* actions, double* rew, uint8_t* done_out,
                                        uint8_t* trunc_out, uint8_t* listed_out, uint8_t* reset_out, int* reset_list,
                                        int* reset_count, void* obs_out, int env0, int env1, lu8* smem) {
    // The Dev fields are read through a pointer re-derived from the kernarg segment at each phase (ZS_TICK_LAUNDER):
    // read through the kernel's by-value argument, the compiler loads them all up front and keeps them in SGPRs
    // for the whole tick (458 SGPR spills into VGPR lanes at G = 8, each use a v_readlane).
    const Dev* dp = ZS_TICK_LAUNDER ? zs_launder_dev(d0) : &d0;
#if ZS_TICK_LAUNDER
#define ZS_RELOAD_DEV() dp = zs_launder_dev(d0)
#else
#define ZS_RELOAD_DEV() (void)0
#endif
    constexpr int NE = 64 / G;
#ifndef ZS_DIAG_STOP
#define ZS_DIAG_STOP 0  // diagnostic builds only: end the tick after phase k (1 stage-in ... 5 MT refill; 6-10 inside the execution; 11-12 in the leader part)
#endif
#define ZS_STOP_AFTER(k) \
    if (ZS_DIAG_STOP == (k)) return
    const int lane = threadIdx.x & 63, g = lane / G, j = lane - g * G;
    const int base = env0 + wg * NE, e = base + g, N = dp->N, E = dp->E, A = dp->A;
    const bool active = e < env1;
    const bool leader = j == 0;
    const TickLayout L = tick_layout(NE, E, dp->DW, dp->rw_cap, dp->cand_cap, dp->lists_cap, A, dp->fobs ? dp->obsl.bytes + 4 * dp->obs_stat : 0);
    lu32* lst = (lu32*)(smem + L.off_lst);
    Grp c;
    c.e = e;
    c.g = g;
    c.j = j;
    c.ne = NE;
    c.misc = (li32*)(smem + L.off_misc);
    c.bm = (lu32*)(smem + L.off_bm);
    c.rw = (lu32*)(smem + L.off_rw);
    c.cand = (lu16*)(smem + L.off_cand);
    c.lpos = (li32*)(smem + L.off_pos);
    c.llife = (li32*)(smem + L.off_life);
    c.ltgt = (li32*)(smem + L.off_tgt);
    c.lweap = (lu8*)(smem + L.off_weap);
    c.lpres = (lu8*)(smem + L.off_pres);
    c.lorder = (lu8*)(smem + L.off_order);
    c.lrank = (lu8*)(smem + L.off_rank);
    c.lkind = (lu8*)(smem + L.off_kind);
    c.lperm = (lu8*)(smem + L.off_perm);
    c.lmoved = (lu8*)(smem + L.off_moved);
    c.lact = (li32*)(smem + L.off_act);
    c.xs = (li32*)(smem + L.off_xs);
    c.lists = (li32*)(smem + L.off_lists);
    if (dp->lists_cap)  // the static spawn lists, staged once per workgroup
        for (int i = lane; i < dp->nps + dp->nzs; i += 64) c.lists[i] = i < dp->nps ? dp->pspawn[i] : dp->zspawn[i - dp->nps];

    STAMP_DECL
    STAMP(0);
    // needs_reset != 0: the env ended at the previous call (or was never reset) and is rebuilt by
    // this call's reset work, possibly concurrently: its state is neither read nor written here,
    // only this call's outputs (as after env.reset()) and the flag.
    int needs_reset = 0, stepping = 0, n_order = 0;
    uint32_t st0 = 0, st = 0;
    int wlen = 0;
    // One round of loads for the flag, the stream state and the first batch of the entity table,
    // scalar rows and bitmap, issued for every active env (a pending env's values go unused), then
    // the LDS stores: one memory wait instead of one per kind of row.
    int32_t vp[4], vl[4];
    uint8_t vw[4], vr[4], vo[4];
    int mval = 0, av = 0;
    uint32_t bmv[8], opw = 0u;
    uint32_t wv[4];  // EARLY: the window's words j, j + G, j + 2G, j + 3G (raw)
    uint64_t pseed = 0, pstep = 0;  // the fused policy's inputs (zs_step_graph)
    // the window of the stream state st: its first word (off, slot, ready) and length
    auto window = [&](uint32_t st_, uint32_t& off, uint32_t& slot, uint32_t& ready) {
        off = st_ & 1023u, slot = (st_ >> 10) & 1u, ready = (st_ >> 11) & 1u;
        if (off >= ZS_MT_N && ready) {
            slot ^= 1u;
            off = 0;
            ready = 0;
        }
        const int maxw = off >= ZS_MT_N ? 0 : (ready ? dp->rw_cap : min(dp->rw_cap, ZS_MT_N - (int)off));
        return min(dp->rw_step, maxw);
    };
    const int nmisc = MISC_N + 2 * A;
    if (active) {
        if (dp->pol_n) {
            pseed = dp->seeds[e];
            pstep = *dp->pol_step;
        } else if (A) {
            av = actions[(size_t)e * A * 3 + min(j, 3 * A - 1)];
        }
        needs_reset = dp->scal[S_NEEDRESET * N + e];
        n_order = dp->scal[S_NORDER * N + e];
        st = dp->rngst[e];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int s = j + u * G;
            if (s < E) {  // slots past E issue nothing (an all-lanes-false batch is skipped)
                vp[u] = dp->pos[EIX(*dp, s, e)];
                vl[u] = dp->life[EIX(*dp, s, e)];
                vw[u] = dp->weapon[EIX(*dp, s, e)];
                vr[u] = dp->present[EIX(*dp, s, e)];
                vo[u] = dp->order[EIX(*dp, s, e)];
            }
        }
        mval = misc_load(*dp, min(j, nmisc - 1), e);
        opw = dp->obst_present[(size_t)e * dp->OW + min(j, max(dp->OW - 1, 0))];
    }
    // occupancy is rebuilt here, not kept in HBM: the map's obstacle cells (static, shared by every env,
    // cache-resident; loaded once per wave, each word stored to all NE envs' rows), minus the obstacles
    // an env has lost, plus its present things
#pragma unroll
    for (int u = 0; u < 8; u++)
        if (64 * u < dp->DW) bmv[u] = dp->obstbits[min(lane + 64 * u, dp->DW - 1)];
    stepping = active && needs_reset == 0;
    if (active && dp->pol_n) {
        // zs_step_graph: the policy's actions for this step (zs_gen_actions' stream), written out to the
        // caller's action buffer as the policy kernel would (envs reset by this call included)
        for (int k = j; k < 3 * A; k += G) {
            const int32_t v = policy_action(pseed, pstep, dp->pol_n, k);
            ((int32_t*)actions)[(size_t)e * A * 3 + k] = v;
            if (stepping) LACT(c, k) = v;
        }
    }
#pragma unroll
    for (int u = 0; u < 8; u++)
        if (64 * u < dp->DW && lane + 64 * u < dp->DW) bcast_row<NE>(c.bm, lane + 64 * u, bmv[u]);
    for (int w = 512 + lane; w < dp->DW; w += 64) bcast_row<NE>(c.bm, w, dp->obstbits[w]);  // maps past 128 x 128
    if (stepping) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int s = j + u * G;
            if (s < E) {
                c.lpos[IX(c, s)] = vp[u];
                c.llife[IX(c, s)] = vl[u];
                c.lweap[IX(c, s)] = vw[u];
                c.lpres[IX(c, s)] = vr[u];
                c.lorder[IX(c, s)] = vo[u];
            }
        }
        if (j < nmisc) MISC(c, j) = mval;
        if (!dp->pol_n) {
            if (j < 3 * A) LACT(c, j) = av;
            for (int k = j + G; k < 3 * A; k += G) LACT(c, k) = actions[(size_t)e * A * 3 + k];
        }
        SX(1);
        // the rest of the entity table (E > 4G) (SoA [slot][N]: this env's column)
        {
            auto ix = [&](int s) { return IX(c, s); };

            for (int b = j + 4 * G; b < E; b += 4 * G) {
                int32_t vp[4], vl[4];
                uint8_t vw[4], vr[4], vo[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    int s = min(b + u * G, E - 1);
                    vp[u] = dp->pos[EIX(*dp, s, e)];
                    vl[u] = dp->life[EIX(*dp, s, e)];
                    vw[u] = dp->weapon[EIX(*dp, s, e)];
                    vr[u] = dp->present[EIX(*dp, s, e)];
                    vo[u] = dp->order[EIX(*dp, s, e)];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    int s = b + u * G;
                    if (s < E) {
                        c.lpos[ix(s)] = vp[u];
                        c.llife[ix(s)] = vl[u];
                        c.lweap[ix(s)] = vw[u];
                        c.lpres[ix(s)] = vr[u];
                        c.lorder[ix(s)] = vo[u];
                    }
                }
            }
        }
        // the rest of the per-env scalars and reward tracker / env.agents rows (more rows than lanes)
        for (int f = j + G; f < nmisc; f += G) MISC(c, f) = misc_load(*dp, f, e);
        // RNG window: the next words of this env's stream, tempered
        uint32_t off, slot, ready;
        int b0 = j;
        wlen = window(st, off, slot, ready);
        if constexpr (EARLY) {
            // the window's first 4G words: issued now, into LDS only once the decisions are made (the first
            // reader is the shuffle), so their round trip, which needs the stream state of round 1, runs
            // under the decisions instead of lengthening the stage-in
            const uint32_t* ringe = dp->ring + (size_t)e * ZS_RING_WORDS;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t q = off + min(j + u * G, max(wlen - 1, 0));
                wv[u] = q < ZS_MT_N ? ringe[slot * ZS_MT_N + q] : ringe[(slot ^ 1u) * ZS_MT_N + q - ZS_MT_N];
            }
            b0 = j + 4 * G;
        }
        const uint32_t* ring = dp->ring + (size_t)e * ZS_RING_WORDS;
        for (int b = b0; b < wlen; b += 8 * G) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                uint32_t q = off + min(b + u * G, wlen - 1);
                v[u] = q < ZS_MT_N ? ring[slot * ZS_MT_N + q] : ring[(slot ^ 1u) * ZS_MT_N + q - ZS_MT_N];
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (b + u * G < wlen) c.rw[IX(c, b + u * G)] = mt_temper(v[u]);
        }
        st0 = st_pack(off, slot, ready);
        SX(2);
    }
    wave_sync();
    if (stepping) {
        // dict-order ranks for closest() tie-breaks
        for (int k = j; k < n_order; k += G) LR(c, LO(c, k)) = (uint8_t)k;
        // the cells of obstacles this env has lost (cleaned up, core.py:121-138) are free
        auto lost = [&](int w, uint32_t pw) {
            const int nb = min(32, dp->O - 32 * w);
            uint32_t gone = ~pw & (nb == 32 ? 0xffffffffu : ((1u << nb) - 1u));
            while (gone) {
                const int32_t op = dp->obst_xy[32 * w + __ffs(gone) - 1];
                gone &= gone - 1;
                const int cell = unpack_y(op) * dp->W + unpack_x(op);
                __hip_atomic_fetch_and(&c.bm[IX(c, cell >> 5)], ~(1u << (cell & 31)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        };
        if (j < dp->OW) lost(j, opw);
        for (int w = j + G; w < dp->OW; w += G) lost(w, dp->obst_present[(size_t)e * dp->OW + w]);
    }
    wave_sync();
    if (stepping) {  // the present things' cells (one may stand where a lost obstacle was)
        for (int s = j; s < E; s += G)
            if (LPR(c, s)) {
                const int32_t p = LP(c, s);
                const int cell = unpack_y(p) * dp->W + unpack_x(p);
                __hip_atomic_fetch_or(&c.bm[IX(c, cell >> 5)], 1u << (cell & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            }
    }
    wave_sync();
    STAMP(1);
    ZS_RELOAD_DEV();
    ZS_STOP_AFTER(1);
    if (stepping) {
        // decisions (start-of-tick state), then the action list of get_actions (core.py:80-101) compacted from
        // them in dict order, when no decision was deferred to the leader (RNG-drawing) or raises:
        // MISC_NMOVED = its length, else -1.  A decision reads only the start-of-tick state.  With 32 or more
        // lanes per env the lanes take the actors by slot class (agents, bots, zombies), so a wave runs each
        // class's code once per pass instead of the agent path in every pass that holds an agent of one of its
        // envs (C4, 54 actors: tick 124.2 -> 120.8 us); with fewer lanes the extra pass costs more than it
        // saves (C3: 82.3 -> 86.4 us; profiles/r05e_ab_decide_by_class.log), and the lanes walk the dict order.
        constexpr bool BYCLASS = G >= 32;
        int nact = 0;
        unsigned long long special = 0ull;
        if constexpr (BYCLASS) {
            for (int b0 = 0; b0 < A; b0 += G) {
                const int s = b0 + j;
                if (s < A && LPR(c, s)) {
                    int kk = K_NONE, tgt = 0;
                    decide_agent(*dp, c, s, kk, tgt);
                    LK(c, s) = (uint8_t)kk;
                    LT(c, s) = tgt;
                }
            }
            for (int b0 = A; b0 < A + dp->P; b0 += G) {
                const int s = b0 + j;
                if (s < A + dp->P && LPR(c, s)) {
                    int kk = K_NONE, tgt = 0;
                    decide_bot(*dp, c, s, false, kk, tgt);
                    LK(c, s) = (uint8_t)kk;
                    LT(c, s) = tgt;
                }
            }
            for (int b0 = A + dp->P; b0 < E; b0 += G) {
                const int s = b0 + j;
                if (s < E && LPR(c, s)) {
                    int kk = K_NONE, tgt = 0;
                    decide_zombie(*dp, c, s, false, kk, tgt);
                    LK(c, s) = (uint8_t)kk;
                    LT(c, s) = tgt;
                }
            }
            wave_sync();
        }
        for (int b0 = 0; b0 < n_order; b0 += G) {
            const int k = b0 + j;
            int s = 0, kk = K_NONE, tgt = 0;
            if (k < n_order) {
                s = LO(c, k);
                if constexpr (BYCLASS) {
                    kk = LK(c, s);
                } else {
                    decide(*dp, c, s, actions, false, kk, tgt);
                    LK(c, s) = (uint8_t)kk;
                    LT(c, s) = tgt;
                }
            }
            const bool keep = kk == K_MOVE || kk == K_ATTACK || kk == K_HEAL;
            const unsigned long long sb = __ballot(kk == K_DEFER || kk == K_RAISE);
            const unsigned long long kb = __ballot(keep);
            const unsigned long long gk = G == 64 ? kb : (kb >> (g * G)) & ((1ull << G) - 1ull);
            special |= G == 64 ? sb : (sb >> (g * G)) & ((1ull << G) - 1ull);
            if (keep) LPE(c, nact + __popcll(gk & ((1ull << j) - 1ull))) = (uint8_t)s;
            nact += __popcll(gk);
        }
        if (j == 0) MISC(c, MISC_NMOVED) = special ? -1 : nact;
        if constexpr (EARLY) {  // the window's first 4G words (issued at the stage-in)
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (j + u * G < wlen) c.rw[IX(c, j + u * G)] = mt_temper(wv[u]);
        }
    }
    wave_sync();
    STAMP(2);
    ZS_RELOAD_DEV();
    ZS_STOP_AFTER(2);
    if (active && leader && !stepping) {  // this call is the env's reset; outputs as after env.reset()
        int nr = dp->reward_mode == ZS_REWARD_SINGLE ? 1 : A;
        for (int a = 0; a < nr; a++) rew[(size_t)e * nr + a] = 0.0;
        done_out[e] = 0;
        trunc_out[e] = 0;
        if (listed_out)
            for (int a = 0; a < A; a++) listed_out[(size_t)e * A + a] = 1;
        if (reset_out) reset_out[e] = 1;
        dp->scal[S_NEEDRESET * N + e] = 0;
        lst[g] = 1u << 11;  // no MT refill for this env here
    }
    // the stream window, in every lane of a stepping env (the lanes' draws and the leader's continue it)
    c.st0 = st0;
    c.wpos = 0;
    c.wlen = wlen;
    // the shuffle and execution by the env's lanes when no decision was deferred to the leader (grp_execute)
    bool par = false;
    int nm0 = 0;
    if (stepping && dp->par_exec) {
        const int nact = MISC(c, MISC_NMOVED);
        if (nact >= 0 && nact <= 2 * G) {
            int pos = 0, odirty = 0;
            grp_shuffle<G>(*dp, c, nact, pos);
            if (ZS_DIAG_STOP != 6) grp_execute<G>(*dp, c, nact, pos, nm0, odirty);
            if (dp->alog) {  // the executed actions in execution order (drop-in views)
                int32_t* al = dp->alog + (size_t)e * dp->E * 2;
                for (int k = j; k < nact; k += G) {
                    const int s = LPE(c, k);
                    al[2 * k] = s | (LK(c, s) << 8);
                    al[2 * k + 1] = LT(c, s);
                }
                if (j == 0) dp->alog_n[e] = nact;
            }
            for (int q = j; q < nm0; q += G) LR(c, LM(c, q)) = 255;  // re-inserted at the end of the dict
            if (odirty && j == 0) MISC(c, MISC_ODIRTY) = 1;
            c.wpos = pos;
            par = true;
        }
    }
    wave_sync();
    STAMP(3);
    ZS_RELOAD_DEV();
    ZS_STOP_AFTER(3);
    if (ZS_DIAG_STOP >= 6 && ZS_DIAG_STOP <= 10) return;  // the execution's own stop points (6: the shuffle only, 7-10 in grp_execute)
    if (leader && stepping) {
        c.n_order = n_order;
        c.t = MISC(c, MISC_T) + 1;
        c.deaths = MISC(c, MISC_DEATHS);
        c.zd = MISC(c, MISC_ZD);
        c.epsteps = MISC(c, MISC_EPSTEPS);
        c.prevzd = MISC(c, MISC_PREVZD);
        c.serial = MISC(c, MISC_SERIAL);
        c.odirty = MISC(c, MISC_ODIRTY);
        if (par) {  // every action executed by the lanes: what the leader's part hands on
            MISC(c, MISC_NMOVED) = nm0;
            MISC(c, MISC_NORD) = c.n_order;
        } else {
            XEV(1);
            env_step_leader(*dp, c, actions, rew, done_out, trunc_out, listed_out);
        }
    }
    wave_sync();
    ZS_STOP_AFTER(11);  // diagnostic builds: 11 after the leader's first part, 12 after the group's cleanup
    env_cleanup_group<G>(*dp, c, stepping);
    wave_sync();
    ZS_STOP_AFTER(12);
    if (leader && stepping) {
        if (MISC(c, MISC_NMOVED) >= 0) env_step_leader_b(*dp, c, rew, done_out, trunc_out, listed_out);
        if (c.fin && (dp->flags & ZS_FLAG_AUTORESET)) {
            needs_reset = 1;
            // rebuilt by the next call's reset work; a list holds each env at most once, so an index
            // past N means the counter was not zeroed for this call: never written out of bounds
            const int k = atomicAdd(reset_count, 1);
            if ((unsigned)k < (unsigned)N) reset_list[k] = e;
        }
        if (c.respawn) {  // k_respawn, after this launch
            const int k = atomicAdd(dp->resp_count, 1);
            if ((unsigned)k < (unsigned)N) dp->resp_list[k] = e;
        }
        if (reset_out) reset_out[e] = 0;
        MISC(c, MISC_T) = c.t;
        MISC(c, MISC_DEATHS) = c.deaths;
        MISC(c, MISC_ZD) = c.zd;
        MISC(c, MISC_EPSTEPS) = c.epsteps;
        MISC(c, MISC_PREVZD) = c.prevzd;
        MISC(c, MISC_SERIAL) = c.serial;
        MISC(c, MISC_ODIRTY) = c.odirty;
        dp->scal[S_NORDER * N + e] = c.n_order;
        dp->scal[S_NEEDRESET * N + e] = needs_reset;
        uint32_t stf = st_advance(c.st0, c.wpos);
        dp->rngst[e] = stf;
        lst[g] = stf;
    }
    wave_sync();
    // the multi-agent rewards by the agents' lanes (env_step_leader_b ran: the scratch row is its end-reward code)
    if (stepping && dp->reward_mode == ZS_REWARD_MULTI && MISC(c, MISC_NMOVED) >= 0) multi_rewards(*dp, c, rew, listed_out);
    wave_sync();
    STAMP(4);
    ZS_RELOAD_DEV();
    ZS_STOP_AFTER(4);
    // the MT refill first: its loads do not wait behind the stage-out's stores (one vmcnt for both)
    coop_refill(*dp, base, min(NE, env1 - base), lst, (lu32*)(smem + L.off_bm));
    STAMP(5);
    ZS_RELOAD_DEV();
    ZS_STOP_AFTER(5);
    if (stepping) {
        for (int s = j; s < E; s += G) {
            dp->pos[EIX(*dp, s, e)] = LP(c, s);
            dp->life[EIX(*dp, s, e)] = LL(c, s);
            dp->weapon[EIX(*dp, s, e)] = LW(c, s);
            dp->present[EIX(*dp, s, e)] = LPR(c, s);
            dp->order[EIX(*dp, s, e)] = LO(c, s);
        }
        for (int f = j; f < MISC_N + 2 * A; f += G) misc_store(*dp, f, e, MISC(c, f));
    }
    wave_sync();
    STAMP(6);
    ZS_RELOAD_DEV();
    // observations of the envs ticked here (envs reset by this call get theirs from the reset work):
    // the whole wave encodes one env at a time, its image aliasing the dead tick region
    if (dp->fobs && obs_out) {
        const unsigned long long stepmask = __ballot(stepping && leader);  // bit g * G per stepping env
        lu8* img = (lu8*)(smem + L.off_region);
        lu32* st = dp->obs_stat ? (lu32*)(smem + L.off_region + dp->obsl.bytes) : nullptr;
        if (st && stepmask) obs_stage_static(*dp, st, lane, 64);
        for (int g2 = 0; g2 < NE; g2++) {
            if (!((stepmask >> (g2 * G)) & 1ull)) continue;
            obs_build(*dp, dp->obsl, img, base + g2, [&](int s, int& p, int& lf, int& wp, int& pr) {
                p = c.lpos[s * NE + g2];
                lf = c.llife[s * NE + g2];
                wp = c.lweap[s * NE + g2];
                pr = c.lpres[s * NE + g2];
            });
            obs_stream_any(*dp, dp->obsl, st, img, obs_out, base + g2);
            wave_sync();
        }
    }
    STAMP(7);
#undef ZS_RELOAD_DEV
#undef ZS_STOP_AFTER
}

// Dev is the first argument: tick_wg reloads it from kernarg offset 0 (zs_launder_dev's contract)
template <int G, int W = ZS_STEP_WAVES, bool EARLY = false>
__global__ void __launch_bounds__(64, W) k_tick(Dev d, const int32_t* actions, double* rew, uint8_t* done_out,
                                             uint8_t* trunc_out, uint8_t* listed_out, uint8_t* reset_out,
                                             int* reset_list, int* reset_count, void* obs_out, int env0, int env1) {
    extern __shared__ __align__(16) uint8_t smem[];
    tick_wg<G, EARLY>(d, xcd_remap(blockIdx.x, gridDim.x), actions, rew, done_out, trunc_out, listed_out, reset_out, reset_list,
               reset_count, obs_out, env0, env1, (lu8*)smem);
}
