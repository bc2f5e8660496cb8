// zs_reset.hpp — k_reset: Game.__initialize_world__ (game.py:151-169) for one env per wave.
//
// A reset is the longest serial RNG consumer of the hot path: each spawn_in_random
// (core.py:40-66) filters the candidate cells and Fisher-Yates-shuffles ALL of them
// (bridge64: 40 player + 232 zombie cells, ~400 MT words; maps without zombie spawns:
// every free cell).  Here the whole wave works on one env:
//   * the candidate filter is a ballot compaction over 64 cells at a time;
//   * the MT stream is held one word per lane; each randbelow (random.py:239-249) is
//     one ballot over "lane >= pos && (word >> (32-k)) < n" — the first set bit is the
//     accepted word, so rejection sampling costs no serial memory round trips;
//   * when the block of 624 words runs out the wave twists the next one cooperatively.
// Envs to reset come from a device work list written by k_tick (next-step autoreset) or
// from an env mask (zs_reset).
#pragma once
#include "zs_tick.hpp"
#include "zs_wave_rng.hpp"

struct ResetLds {
    lu32* bm;       // occupancy bitmap [DW]
    lu32* cand;     // candidate cells [ncand]
    li32* lpos;     // [E]
    li32* llife;
    lu8* lweap;
    lu8* lpres;
    lu8* lorder;
    lu8* lslots;    // slots being spawned
    li32* lists;    // static spawn lists (player then zombie), or unused
    lu32* jbuf;     // draw results [max(E, 8)]
    lu32* tw;
};

// the twist buffer doubles as the observation image of the env just rebuilt (obs_bytes)
__host__ __device__ inline int reset_lds_bytes(int E, int DW, int ncand, int lists_cap, int obs_bytes = 0) {
    int o = DW * 4 + ncand * 4 + 2 * E * 4 + 4 * E + lists_cap * 4 + (E + 8) * 4;
    o = ((o + 15) / 16) * 16;
    return o + (obs_bytes > 2 * ZS_MT_N * 4 ? obs_bytes : 2 * ZS_MT_N * 4);
}

__device__ __forceinline__ bool rbm_test(const ResetLds& L, int cell) { return (L.bm[cell >> 5] >> (cell & 31)) & 1u; }

// World.spawn_in_random (core.py:40-66) for k slots in L.lslots[0..k): ballot-compacted
// candidate filter, Fisher-Yates whose first k iterations swap (the popped tail) and whose
// remaining iterations only consume their draws.  Returns the number of things placed.
__device__ __forceinline__ int wave_spawn(const Dev& d, const ResetLds& L, WaveRng& r, int e, int k, int which,
                                          int nlist, int& n_order, int& serial) {
    const int lane = threadIdx.x & 63;
    const int total = nlist ? nlist : d.W * d.H;
    int n = 0;
    for (int b = 0; b < total; b += 64) {
        int i = b + lane;
        int cell = -1;
        if (i < total) {
            if (nlist) {
                int32_t p = d.rlists_cap ? L.lists[(which ? d.nps : 0) + i] : (which ? d.zspawn[i] : d.pspawn[i]);
                cell = unpack_y(p) * d.W + unpack_x(p);
            } else {
                cell = (i % d.H) * d.W + i / d.H;  // x-major (core.py:45-47)
            }
        }
        bool fr = cell >= 0 && !rbm_test(L, cell);
        unsigned long long m = __ballot(fr);
        if (fr) L.cand[n + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)cell;
        n += __popcll(m);
    }
    wave_sync();
    // random.shuffle: for i = n-1 .. 1, j = _randbelow(i+1), swap.  Iterations i >= n-k decide the
    // k popped cells; the rest only consume their draws.
    const int ndraw = max(n - 1, 0), nswap = min(k, ndraw);
    wave_draws(r, n, 1, ndraw, nswap, [&](int t, uint32_t v) { L.jbuf[t] = v; });
    int placed = min(k, n);
    for (int m = lane; m < placed; m += 64) {
        // the m-th popped cell: position n - 1 - m after the first nswap swaps, traced back through them
        int q = n - 1 - m;
        for (int t = nswap - 1; t >= 0; t--) {
            const int i = n - 1 - t, jt = (int)L.jbuf[t];
            q = q == i ? jt : (q == jt ? i : q);
        }
        int s = L.lslots[m];
        int cell = (int)L.cand[q];
        L.lpos[s] = pack_xy(cell % d.W, cell / d.W);
        L.lpres[s] = 1;
        __hip_atomic_fetch_or(&L.bm[cell >> 5], 1u << (cell & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        L.lorder[n_order + m] = (uint8_t)s;
        d.serial[EIX(d, s, e)] = (uint32_t)(serial + m + 1);
    }
    n_order += placed;
    serial += placed;
    wave_sync();
    return placed;
}

// end of a wave's use of the stream: the next block twisted (k_tick's window needs it ready),
// twisted slots written back; returns the stream state to store
__device__ __forceinline__ uint32_t wave_rng_finish(WaveRng& r) {
    uint32_t stf = st_advance(r.st, r.pos);
    if (!((stf >> 11) & 1u)) {
        wave_twist(r, (stf >> 10) & 1u);
        stf |= 1u << 11;
    }
    wave_rng_flush(r);
    return stf;
}

// The Dev fields are read through a pointer re-derived from the kernarg segment at each phase (as tick_wg
// does): read through the kernel's by-value argument they are loaded once and held in SGPRs across the
// whole rebuild, which spills.  The kernels calling this take their Dev as the first argument.
#ifndef ZS_RESET_LAUNDER
#define ZS_RESET_LAUNDER 1
#endif
#if ZS_RESET_LAUNDER
#define ZS_RST_RELOAD() dp = zs_launder_dev(d0)
#else
#define ZS_RST_RELOAD() (void)0
#endif
__device__ __forceinline__ void reset_env_wave(const Dev& d0, const ResetLds& L, int e, int list_mode, int* err_out) {
    const Dev* dp = ZS_RESET_LAUNDER ? zs_launder_dev(d0) : &d0;
    const int lane = threadIdx.x & 63, N = dp->N, E = dp->E, A = dp->A, P = dp->P;
    RST_DECL
    RST(0);
    const uint32_t st_in = dp->rngst[e];
    const int serial0 = dp->scal[S_SERIAL * N + e];
    // the env's ring (both slots, independent of st_in) in the same round of loads as the rows below
    WaveRng r;
    r.ring = dp->ring + (size_t)e * ZS_RING_WORDS;
    r.lr = L.tw;
    uint32_t rv[WR_STAGE_K];
    wave_rng_fetch(r, rv);
    // lane l's player (agents [0, A), bots [A, A + P)): its configured weapon / bot type
    const int wsel = lane < A ? dp->agent_weapons[lane] : lane < A + P ? dp->bot_types[lane - A] : 0;
    // new World: the map's obstacles (all present, HP carried over), no things, no decoration
    for (int w = lane; w < dp->DW; w += 64) {
        L.bm[w] = dp->obstbits[w];
        dp->dead[(size_t)e * dp->DW + w] = 0;
    }
    if (lane == 0) dp->dead_dirty[e] = 0u;
    int nonpos = 0;
    for (int w = lane; w < dp->OW; w += 64) {
        int nb = min(32, dp->O - 32 * w);
        dp->obst_present[(size_t)e * dp->OW + w] = nb == 32 ? 0xffffffffu : ((1u << nb) - 1u);
        nonpos |= dp->obst_nonpos[(size_t)e * dp->OW + w] != 0;
    }
    for (int s = lane; s < E; s += 64) {
        L.lpres[s] = 0;
        L.lpos[s] = dp->pos[EIX(*dp, s, e)];
        L.llife[s] = dp->life[EIX(*dp, s, e)];
        L.lweap[s] = dp->weapon[EIX(*dp, s, e)];
    }
    const int odirty = __ballot(nonpos) != 0ull;
    wave_rng_put(r, rv);
    rng_block_load(r, st_in);
    RST(1); ZS_RST_RELOAD();
    // players: Player() picks a random weapon unless its module gives one (things.py:113-116);
    // agents: WeaponFactory.create_player_weapon (weapons.py:28-45).  Each random pick is one
    // _randbelow(5), in bots-then-agents order.
    if (A + P <= 64) {  // one lane per player: the random picks ranked bots first, then agents
        const bool rnd = lane < A ? wsel == ZS_WEAPON_RANDOM
                                  : lane < A + P && wsel != ZS_BOT_TERMINATOR && wsel != ZS_BOT_SNIPER;
        const unsigned long long rb = __ballot(rnd);
        const unsigned long long bots = ((A + P == 64 ? ~0ull : (1ull << (A + P)) - 1ull) >> A) << A;
        const int rank = lane >= A ? __popcll(rb & bots & ((1ull << lane) - 1ull))
                                   : __popcll(rb & bots) + __popcll(rb & ((1ull << lane) - 1ull));
        const int nrw = __popcll(rb);
        if (nrw) wave_draws(r, 5, 0, nrw, nrw, [&](int t, uint32_t v) { L.jbuf[t] = v; });
        if (lane < A + P) {
            int w;
            if (lane < A) {  // WeaponFactory: choice([Knife(), Axe(), Gun(), Rifle(), Shotgun()]) when random
                const int k = rnd ? (int)L.jbuf[rank] : 0;
                w = !rnd ? wsel : k == 0 ? ZS_WEAPON_KNIFE : k == 1 ? ZS_WEAPON_AXE : k == 2 ? ZS_WEAPON_GUN
                                : k == 3 ? ZS_WEAPON_RIFLE : ZS_WEAPON_SHOTGUN;
            } else if (wsel == ZS_BOT_TERMINATOR) {  // terminator.py:40-42
                w = ZS_WEAPON_SHOTGUN;
            } else if (wsel == ZS_BOT_SNIPER) {      // sniper.py:22-24
                w = ZS_WEAPON_RIFLE;
            } else {                                 // choice([Gun, Shotgun, Rifle, Knife, Axe])
                const int k = (int)L.jbuf[rank];
                w = k == 0 ? ZS_WEAPON_GUN : k == 1 ? ZS_WEAPON_SHOTGUN : k == 2 ? ZS_WEAPON_RIFLE
                    : k == 3 ? ZS_WEAPON_KNIFE : ZS_WEAPON_AXE;
            }
            L.lweap[lane] = (uint8_t)w;
            L.llife[lane] = 100;
        }
    } else {
    int nrw = 0;
    for (int p = 0; p < P; p++) nrw += dp->bot_types[p] != ZS_BOT_TERMINATOR && dp->bot_types[p] != ZS_BOT_SNIPER;
    for (int a = 0; a < A; a++) nrw += dp->agent_weapons[a] == ZS_WEAPON_RANDOM;
    if (nrw) wave_draws(r, 5, 0, nrw, nrw, [&](int t, uint32_t v) { L.jbuf[t] = v; });
    if (lane == 0) {
        int t = 0;
        for (int p = 0; p < P; p++) {
            int bt = dp->bot_types[p], w;
            if (bt == ZS_BOT_TERMINATOR) w = ZS_WEAPON_SHOTGUN;  // terminator.py:40-42
            else if (bt == ZS_BOT_SNIPER) w = ZS_WEAPON_RIFLE;   // sniper.py:22-24
            else {                                               // choice([Gun, Shotgun, Rifle, Knife, Axe])
                int k = (int)L.jbuf[t++];
                w = k == 0 ? ZS_WEAPON_GUN : k == 1 ? ZS_WEAPON_SHOTGUN : k == 2 ? ZS_WEAPON_RIFLE : k == 3 ? ZS_WEAPON_KNIFE : ZS_WEAPON_AXE;
            }
            L.lweap[A + p] = (uint8_t)w;
            L.llife[A + p] = 100;
        }
        for (int a = 0; a < A; a++) {
            int w = dp->agent_weapons[a];
            if (w == ZS_WEAPON_RANDOM) {  // choice([Knife(), Axe(), Gun(), Rifle(), Shotgun()])
                int k = (int)L.jbuf[t++];
                w = k == 0 ? ZS_WEAPON_KNIFE : k == 1 ? ZS_WEAPON_AXE : k == 2 ? ZS_WEAPON_GUN : k == 3 ? ZS_WEAPON_RIFLE : ZS_WEAPON_SHOTGUN;
            }
            L.lweap[a] = (uint8_t)w;
            L.llife[a] = 100;
        }
    }
    }
    wave_sync();
    int n_order = 0, serial = serial0;
    int rc = ZS_OK;
    RST(2); ZS_RST_RELOAD();
    // spawn_players, spawn_agents (game.py:181-187): fail_if_cant=True
    for (int i = lane; i < P; i += 64) L.lslots[i] = (uint8_t)(A + i);
    wave_sync();
    if (wave_spawn(*dp, L, r, e, P, 0, dp->nps, n_order, serial) < P) rc = ZS_ENOSPACE;
    if (rc == ZS_OK) {
        for (int i = lane; i < A; i += 64) L.lslots[i] = (uint8_t)i;
        wave_sync();
        if (wave_spawn(*dp, L, r, e, A, 0, dp->nps, n_order, serial) < A) rc = ZS_ENOSPACE;
    }
    RST(3); ZS_RST_RELOAD();
    if (rc == ZS_OK) {
        // spawn_zombies(initial) (game.py:189-194): Zombie() draws randint(50, 100) first
        int nz = dp->initial_zombies;
        for (int b0 = 0; b0 < nz; b0 += dp->E + 8) {  // randint(50, 100) = 50 + _randbelow(51) each
            int cnt = min(nz - b0, dp->E + 8);
            wave_draws(r, 51, 0, cnt, cnt, [&](int t, uint32_t v) { L.jbuf[t] = v; });
            for (int i = lane; i < cnt; i += 64) {
                L.llife[A + P + b0 + i] = 50 + (int)L.jbuf[i];
                L.lweap[A + P + b0 + i] = ZS_WEAPON_CLAWS;
                L.lslots[b0 + i] = (uint8_t)(A + P + b0 + i);
            }
            wave_sync();
        }
        RST(4); ZS_RST_RELOAD();
        wave_spawn(*dp, L, r, e, nz, 1, dp->nzs, n_order, serial);
        RST(5);
    } else if (lane == 0 && err_out) {
        atomicMax(err_out, rc);
    }
    RST(6); ZS_RST_RELOAD();
    const uint32_t stf = wave_rng_finish(r);
    // write the new world back
    for (int s = lane; s < E; s += 64) {
        dp->pos[EIX(*dp, s, e)] = L.lpos[s];
        dp->life[EIX(*dp, s, e)] = L.llife[s];
        dp->weapon[EIX(*dp, s, e)] = L.lweap[s];
        dp->present[EIX(*dp, s, e)] = L.lpres[s];
        dp->order[EIX(*dp, s, e)] = L.lorder[s];
    }
    for (int a = lane; a < A; a += 64) {  // reward_tracker.reset / env.agents = possible_agents
        dp->prev_life[(size_t)a * N + e] = L.llife[a];
        dp->listed[(size_t)a * N + e] = 1;
    }
    if (lane == 0) {
        dp->scal[S_T * N + e] = -1;
        dp->scal[S_DEATHS * N + e] = 0;
        dp->scal[S_ZD * N + e] = 0;
        dp->scal[S_EPSTEPS * N + e] = 0;
        dp->scal[S_NORDER * N + e] = n_order;
        dp->scal[S_PREVZD * N + e] = 0;
        dp->scal[S_SERIAL * N + e] = serial;
        dp->scal[S_ODIRTY * N + e] = odirty;
        // list mode (autoreset): the env stays pending; the tick of this same call reports it as
        // reset and clears the flag (it never reads this env's state).  Mask mode: done now.
        if (!list_mode) dp->scal[S_NEEDRESET * N + e] = 0;
        dp->rngst[e] = stf;
        if (dp->dlog_n) dp->dlog_n[e] = 0;  // a reset removes nothing and executes nothing (ZS_FLAG_DEATH_LOG)
        if (dp->alog_n) dp->alog_n[e] = 0;
    }
    wave_sync();
    RST(7);
}

// the reset work's LDS image (reset_lds_bytes), the static spawn lists staged when they fit
__device__ __forceinline__ ResetLds reset_lds_carve(const Dev& d, uint8_t* smem, bool stage_lists = true) {
    ResetLds L;
    int o = 0;
    L.bm = (lu32*)(smem + o);
    o += d.DW * 4;
    L.cand = (lu32*)(smem + o);
    o += d.ncand * 4;
    L.lpos = (li32*)(smem + o);
    o += d.E * 4;
    L.llife = (li32*)(smem + o);
    o += d.E * 4;
    L.lweap = (lu8*)(smem + o);
    o += d.E;
    L.lpres = (lu8*)(smem + o);
    o += d.E;
    L.lorder = (lu8*)(smem + o);
    o += d.E;
    L.lslots = (lu8*)(smem + o);
    o += d.E;
    L.lists = (li32*)(smem + o);
    o += d.rlists_cap * 4;
    L.jbuf = (lu32*)(smem + o);
    o += (d.E + 8) * 4;
    o = ((o + 15) / 16) * 16;
    L.tw = (lu32*)(smem + o);
    if (d.rlists_cap && stage_lists)
        for (int i = threadIdx.x & 63; i < d.nps + d.nzs; i += 64) L.lists[i] = i < d.nps ? d.pspawn[i] : d.zspawn[i - d.nps];
    wave_sync();
    return L;
}

// The reset work of workgroup `wg` of `nwg`.  list_mode: envs list[0..*count) (next-step
// autoreset; the list holds exactly the pending envs, see zs_reset's list filter).  Otherwise
// every env with mask[e] (all if mask == NULL).
__device__ __forceinline__ void reset_role(const Dev& d, int list_mode, const int* list, const int* count,
                                           const uint8_t* mask, int* err_out, int wg, int nwg, void* obs_out) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int n = list_mode ? min(*count, d.N) : d.N;
    if (wg >= n) return;
    const ResetLds L = reset_lds_carve(d, smem);
    for (int idx = wg; idx < n; idx += nwg) {
        int e = list_mode ? list[idx] : idx;
        if (!list_mode && mask && !mask[e]) continue;
        reset_env_wave(d, L, e, list_mode, err_out);
        if (obs_out) {  // fobs: the new world's observations, the image aliasing the twist buffer
            wave_sync();
            lu8* img = (lu8*)L.tw;
            lu32* st = d.obs_stat ? (lu32*)((lu8*)L.tw + d.obsl.bytes) : nullptr;
            if (st) obs_stage_static(d, st, threadIdx.x & 63, 64);
            obs_build(d, d.obsl, img, e, [&](int s, int& p, int& lf, int& wp, int& pr) {
                p = L.lpos[s];
                lf = L.llife[s];
                wp = L.lweap[s];
                pr = L.lpres[s];
            });
            obs_stream_any(d, d.obsl, st, img, obs_out, e);
            wave_sync();
        }
    }
}

// the non-template kernels are compiled in k_reset.hip only
#ifdef ZS_DEFINE_RESET_KERNELS
// Dev is the first argument (zs_launder_dev's contract: reset_env_wave reloads it from kernarg offset 0)
__global__ void __launch_bounds__(64, ZS_RESET_WAVES) k_reset(Dev d, int list_mode, const int* list, const int* count,
                                              const uint8_t* mask, int* err_out, void* obs_out) {
    reset_role(d, list_mode, list, count, mask, err_out, blockIdx.x, gridDim.x, obs_out);
}
#endif

// ---------------------------------------------------------------------------
// k_respawn: Game.spawn_zombies_to_maintain_minimum (game.py:196-201) for the envs whose tick
// deferred it (d.defer_respawn: long candidate lists, e.g. city128's 439 zombie spawns or every
// cell of city_for_safehouse).  One wave per env continues the env's stream where the tick left
// it: randint(50, 100) per new Zombie (things.py:61-68), then World.spawn_in_random's shuffle
// (core.py:40-66) as wave work (wave_spawn), new zombies appended to the dict order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void respawn_env_wave(const Dev& d0, const ResetLds& L, int e) {
    const Dev* dp = ZS_RESET_LAUNDER ? zs_launder_dev(d0) : &d0;
    const int lane = threadIdx.x & 63, N = dp->N, E = dp->E, Z0 = dp->A + dp->P;
    RST_DECL
    RST(0);
#ifdef ZS_STAMPS
    if (lane == 0 && blockIdx.x < ZS_STAMP_WGS) g_stamp_wg[blockIdx.x * ZS_NPHASE + 19] += 1;  // respawns (slot 19)
#endif
    WaveRng r;
    r.ring = dp->ring + (size_t)e * ZS_RING_WORDS;
    r.lr = L.tw;
    // one round of loads for all the respawn reads: the env's ring (both slots) and stream state, its
    // counters, entity rows and obstacle-present words, the zombie spawn list, the static bitmap
    uint32_t rv[WR_STAGE_K];
    wave_rng_fetch(r, rv);
    const uint32_t st_in = dp->rngst[e];
    const int n0 = dp->scal[S_NORDER * N + e], serial0 = dp->scal[S_SERIAL * N + e];
    const int sl = min(lane, E - 1);
    const int32_t vp = dp->pos[EIX(*dp, sl, e)], vl = dp->life[EIX(*dp, sl, e)];
    const uint8_t vw = dp->weapon[EIX(*dp, sl, e)], vr = dp->present[EIX(*dp, sl, e)], vo = dp->order[EIX(*dp, sl, e)];
    uint32_t opv[2];
#pragma unroll
    for (int u = 0; u < 2; u++)
        if (64 * u < dp->OW) opv[u] = dp->obst_present[(size_t)e * dp->OW + min(lane + 64 * u, dp->OW - 1)];
    int32_t zl[8];  // k_respawn stages only the zombie spawn list (reset_lds_carve's stage_lists false)
    if (dp->rlists_cap) {
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (64 * u < dp->nzs) zl[u] = dp->zspawn[min(lane + 64 * u, dp->nzs - 1)];
    }
    stage_in(dp->obstbits, dp->DW, lane, 64, L.bm, [](int w) { return w; });
    if (dp->rlists_cap) {
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (64 * u < dp->nzs && lane + 64 * u < dp->nzs) L.lists[dp->nps + lane + 64 * u] = zl[u];
        for (int i = 512 + lane; i < dp->nzs; i += 64) L.lists[dp->nps + i] = dp->zspawn[i];
    }
    if (lane < E) {
        L.lpos[lane] = vp;
        L.llife[lane] = vl;
        L.lweap[lane] = vw;
        L.lpres[lane] = vr;
        L.lorder[lane] = vo;
    }
    for (int s = 64 + lane; s < E; s += 64) {
        L.lpos[s] = dp->pos[EIX(*dp, s, e)];
        L.llife[s] = dp->life[EIX(*dp, s, e)];
        L.lweap[s] = dp->weapon[EIX(*dp, s, e)];
        L.lpres[s] = dp->present[EIX(*dp, s, e)];
        L.lorder[s] = dp->order[EIX(*dp, s, e)];
    }
    RST(1); ZS_RST_RELOAD();
    // occupancy (as k_tick rebuilds it): the map's obstacle cells minus the lost obstacles, then the
    // present things
    wave_sync();
    auto lost = [&](int w, uint32_t pw) {
        const int nb = min(32, dp->O - 32 * w);
        uint32_t gone = ~pw & (nb == 32 ? 0xffffffffu : ((1u << nb) - 1u));
        while (gone) {
            const int32_t op = dp->obst_xy[32 * w + __ffs(gone) - 1];
            gone &= gone - 1;
            const int cell = unpack_y(op) * dp->W + unpack_x(op);
            __hip_atomic_fetch_and(&L.bm[cell >> 5], ~(1u << (cell & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
#pragma unroll
    for (int u = 0; u < 2; u++)
        if (lane + 64 * u < dp->OW) lost(lane + 64 * u, opv[u]);
    for (int w = 128 + lane; w < dp->OW; w += 64) lost(w, dp->obst_present[(size_t)e * dp->OW + w]);
    wave_sync();
    for (int s = lane; s < E; s += 64)
        if (L.lpres[s]) {
            const int cell = unpack_y(L.lpos[s]) * dp->W + unpack_x(L.lpos[s]);
            __hip_atomic_fetch_or(&L.bm[cell >> 5], 1u << (cell & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    wave_rng_put(r, rv);
    rng_block_load(r, st_in);
    RST(2); ZS_RST_RELOAD();
    // Game.spawn_zombies(count): the deficit's Zombie()s go into the free zombie slots, lowest first
    int nz = 0;
    for (int b = Z0; b < E; b += 64) nz += __popcll(__ballot(b + lane < E && L.lpres[b + lane]));
    const int k = max(dp->minimum_zombies - nz, 0);
#ifdef ZS_STAMPS
    if (lane == 0 && k > 0 && blockIdx.x < ZS_STAMP_WGS) g_stamp_wg[blockIdx.x * ZS_NPHASE + 19] += 1ull << 32;  // placing ones
#endif
    int taken = 0;
    for (int b = Z0; b < E && taken < k; b += 64) {
        const int s = b + lane;
        const bool fr = s < E && !L.lpres[s];
        const unsigned long long m = __ballot(fr);
        const int rk = taken + __popcll(m & ((1ull << lane) - 1ull));
        if (fr && rk < k) L.lslots[rk] = (uint8_t)s;
        taken += __popcll(m);
    }
    wave_sync();
    wave_draws(r, 51, 0, k, k, [&](int t, uint32_t v) {
        const int s = L.lslots[t];
        L.llife[s] = 50 + (int)v;
        L.lweap[s] = ZS_WEAPON_CLAWS;
    });
    int n_order = n0, serial = serial0;
    RST(3); ZS_RST_RELOAD();
    const int placed = wave_spawn(*dp, L, r, e, k, 1, dp->nzs, n_order, serial);
    RST(4); ZS_RST_RELOAD();
    const uint32_t stf = wave_rng_finish(r);
    for (int m = lane; m < k; m += 64) {  // the new zombies (dropped ones keep their drawn life)
        const int s = L.lslots[m];
        dp->pos[EIX(*dp, s, e)] = L.lpos[s];
        dp->life[EIX(*dp, s, e)] = L.llife[s];
        dp->weapon[EIX(*dp, s, e)] = L.lweap[s];
        dp->present[EIX(*dp, s, e)] = L.lpres[s];
    }
    for (int m = n0 + lane; m < n0 + placed; m += 64) dp->order[EIX(*dp, m, e)] = L.lorder[m];
    if (lane == 0) {
        dp->scal[S_NORDER * N + e] = n_order;
        dp->scal[S_SERIAL * N + e] = serial;
        dp->rngst[e] = stf;
    }
    wave_sync();
    RST(5);
}

#ifdef ZS_DEFINE_RESET_KERNELS
// the merged load round needs the registers: at 6 waves per SIMD 244 B of spills, at 4 60 B; at 3 none
// (C4, one box: respawn + gaps 31 us before the merge, 35 at 4 waves, 30 at 3; profiles/r04_ab_respawn.log)
#ifndef ZS_RESPAWN_WAVES
#define ZS_RESPAWN_WAVES 3
#endif
// Dev is the first argument (zs_launder_dev's contract: respawn_env_wave reloads it from kernarg offset 0)
__global__ void __launch_bounds__(64, ZS_RESPAWN_WAVES) k_respawn(Dev d) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int cnt = *d.resp_count, e0 = d.resp_list[blockIdx.x];  // one round trip (grid <= N)
    const int n = min(cnt, d.N);
    if ((int)blockIdx.x >= n) return;
    const ResetLds L = reset_lds_carve(d, smem, false);  // the zombie list: with the env's loads
    for (int idx = blockIdx.x; idx < n; idx += gridDim.x) respawn_env_wave(d, L, idx == (int)blockIdx.x ? e0 : d.resp_list[idx]);
}

// Drop the envs a mask-mode reset just rebuilt from the pending list (src -> dst, dst count
// zeroed by the host); mask == NULL drops all.  Keeps "list == pending envs" exact.
__global__ void __launch_bounds__(256) k_list_filter(const int* src, const int* src_count, int* dst, int* dst_count,
                                                     const uint8_t* mask, int N) {
    if (!mask) return;
    const int n = min(*src_count, N);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        int e = src[i];
        if (!mask[e]) dst[atomicAdd(dst_count, 1)] = e;
    }
}
#endif  // ZS_DEFINE_RESET_KERNELS
