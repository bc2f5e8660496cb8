// engine.hip — MI355X-native batched zombsole step engine (gfx950) and its C ABI.
//
// One lane per env runs the reference's strictly sequential tick
// (World.step, core.py:72-78: decide in dict order -> shuffle -> execute ->
// cleanup, then rewards, respawn, rules) on state staged in LDS; a wave of 64
// lanes steps 64 envs in lock-step.  The MT19937 refill is wave-cooperative
// (3 dependency phases over a 624-word block); observations are produced by
// a separate cell-parallel kernel that streams the int64/int32 planes.
//
// Semantics follow the reference exactly (parity: tests/); every sqrt range
// test of the reference is replaced by its exact integer d^2 equivalent.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "zs_device.hpp"

#define NOTHING ((int)0x80000000)

enum { K_NONE = 0, K_MOVE = 1, K_ATTACK = 2, K_HEAL = 3 };

// adjacent_positions order (utils.py:34-44)
__constant__ int c_adj_dx[4] = {0, 0, 1, -1};
__constant__ int c_adj_dy[4] = {1, -1, 0, 0};

// ---------------------------------------------------------------------------
// per-lane context: the env's entity table lives in LDS as [slot][lane]
// ---------------------------------------------------------------------------
struct Lane {
    int e, lane, wg;
    int32_t* lpos;
    int32_t* llife;
    int32_t* ltgt;
    uint8_t* lweap;
    uint8_t* lpres;
    uint8_t* lorder;
    uint8_t* lrank;
    uint8_t* lkind;
    uint8_t* lperm;
    uint8_t* lmoved;
    Rng rng;
    int n_order;
    int t, deaths, zd, epsteps, prevzd, serial, odirty;
};

#define LP(c, s) (c).lpos[(s) * (c).wg + (c).lane]
#define LL(c, s) (c).llife[(s) * (c).wg + (c).lane]
#define LT(c, s) (c).ltgt[(s) * (c).wg + (c).lane]
#define LW(c, s) (c).lweap[(s) * (c).wg + (c).lane]
#define LPR(c, s) (c).lpres[(s) * (c).wg + (c).lane]
#define LO(c, s) (c).lorder[(s) * (c).wg + (c).lane]
#define LR(c, s) (c).lrank[(s) * (c).wg + (c).lane]
#define LK(c, s) (c).lkind[(s) * (c).wg + (c).lane]
#define LPE(c, s) (c).lperm[(s) * (c).wg + (c).lane]
#define LM(c, s) (c).lmoved[(s) * (c).wg + (c).lane]

__device__ __forceinline__ size_t lds_bytes_per_slot() { return 3 * 4 + 7; }

__device__ __forceinline__ bool in_bounds(const Dev& d, int x, int y) {
    return x >= 0 && y >= 0 && x < d.W && y < d.H;
}

__device__ __forceinline__ bool obst_is_present(const Dev& d, const Lane& c, int oi) {
    return (d.obst_present[(size_t)c.e * d.OW + (oi >> 5)] >> (oi & 31)) & 1u;
}

// World.things.get(position): entity slot (>= 0), obstacle -(index+1), or NOTHING
__device__ __forceinline__ int thing_at(const Dev& d, const Lane& c, int x, int y) {
    if (!in_bounds(d, x, y)) return NOTHING;
    int cell = y * d.W + x;
    int s = (int)d.occ[(size_t)c.e * d.occ_stride + cell] - 1;
    if (s >= 0) return s;
    int oi = d.cellmap[cell];
    if (oi >= 0 && obst_is_present(d, c, oi)) return -(oi + 1);
    return NOTHING;
}

__device__ __forceinline__ int slot_kind(const Dev& d, int s) {
    return s < d.A ? ZS_THING_AGENT : (s < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
}

__device__ __forceinline__ int32_t target_pos(const Dev& d, const Lane& c, int tgt) {
    return tgt >= 0 ? LP(c, tgt) : d.obst_xy[-tgt - 1];
}

__device__ __forceinline__ int target_maxlife(const Dev& d, int tgt) {
    if (tgt >= 0) return 100;  // Zombie / Player / Agent MAX_LIFE (things.py:62,109)
    return d.obst_kind[-tgt - 1] == ZS_THING_BOX ? 10 : 200;
}

__device__ __forceinline__ int target_life(const Dev& d, const Lane& c, int tgt) {
    return tgt >= 0 ? LL(c, tgt) : d.obst_hp[(size_t)c.e * d.O + (-tgt - 1)];
}

__device__ __forceinline__ void set_target_life(const Dev& d, Lane& c, int tgt, int v) {
    if (tgt >= 0) {
        LL(c, tgt) = v;
        return;
    }
    int oi = -tgt - 1;
    d.obst_hp[(size_t)c.e * d.O + oi] = v;
    uint32_t* w = &d.obst_nonpos[(size_t)c.e * d.OW + (oi >> 5)];
    uint32_t bit = 1u << (oi & 31);
    *w = v <= 0 ? (*w | bit) : (*w & ~bit);
    c.odirty = 1;
}

// closest(...) over present slots [s0, s1) \ {excl}: first minimum in dict order
__device__ __forceinline__ int closest_in(const Dev& d, const Lane& c, int fx, int fy, int s0, int s1, int excl) {
    int best = -1, bd = 0, br = 0;
    for (int s = s0; s < s1; s++) {
        if (!LPR(c, s) || s == excl) continue;
        int p = LP(c, s);
        int dd = d2(fx, fy, unpack_x(p), unpack_y(p));
        int rk = LR(c, s);
        if (best < 0 || dd < bd || (dd == bd && rk < br)) {
            best = s;
            bd = dd;
            br = rk;
        }
    }
    return best;
}

// ---------------------------------------------------------------------------
// placement / spawning
// ---------------------------------------------------------------------------
__device__ __forceinline__ void place(const Dev& d, Lane& c, int s, int cell) {
    int x = cell % d.W, y = cell / d.W;
    LP(c, s) = pack_xy(x, y);
    LPR(c, s) = 1;
    d.occ[(size_t)c.e * d.occ_stride + cell] = (uint8_t)(s + 1);
    LO(c, c.n_order) = (uint8_t)s;
    c.n_order++;
    d.serial[(size_t)s * d.N + c.e] = (uint32_t)(++c.serial);
}

// World.spawn_in_random (core.py:40-66) for the k slots listed in LM(c, 0..k).
// Only the first k Fisher-Yates iterations can move the k cells that get popped;
// the remaining iterations are replayed for their RNG draws alone.
__device__ int spawn_in_random(const Dev& d, Lane& c, int k, const int32_t* list, int nlist, int fail_if_cant) {
    int32_t* cand = d.cand + (size_t)c.e * d.ncand;
    int n = 0;
    if (nlist == 0) {  // every cell, x-major (core.py:45-47)
        for (int x = 0; x < d.W; x++)
            for (int y = 0; y < d.H; y++)
                if (thing_at(d, c, x, y) == NOTHING) cand[n++] = y * d.W + x;
    } else {
        for (int i = 0; i < nlist; i++) {
            int32_t p = list[i];
            int x = unpack_x(p), y = unpack_y(p);
            if (thing_at(d, c, x, y) == NOTHING) cand[n++] = y * d.W + x;
        }
    }
    int lim = n - k;
    for (int i = n - 1; i >= 1; i--) {
        int j = rng_below(c.rng, i + 1);
        if (i >= lim) {
            int tmp = cand[i];
            cand[i] = cand[j];
            cand[j] = tmp;
        }
    }
    for (int m = 0; m < k; m++) {
        int s = LM(c, m);
        if (m < n) {
            place(d, c, s, cand[n - 1 - m]);
        } else {
            if (fail_if_cant) return ZS_ENOSPACE;
            for (int q = m; q < k; q++) LPR(c, LM(c, q)) = 0;  // dropped (game.py:192-194)
            return ZS_OK;
        }
    }
    return ZS_OK;
}

// Game.spawn_zombies(count) into the free zombie slots (game.py:189-194); Zombie() draws
// randint(50, 100) for each zombie before the spawn shuffle (things.py:61-68).
__device__ void spawn_zombies(const Dev& d, Lane& c, int count) {
    int k = 0;
    for (int s = d.A + d.P; s < d.E && k < count; s++)
        if (!LPR(c, s)) LM(c, k++) = (uint8_t)s;
    for (int i = 0; i < k; i++) {
        int s = LM(c, i);
        LL(c, s) = rng_int(c.rng, 50, 100);
        LW(c, s) = ZS_WEAPON_CLAWS;
    }
    spawn_in_random(d, c, k, d.zspawn, d.nzs, 0);
}

// ---------------------------------------------------------------------------
// reset: Game.__initialize_world__ (game.py:151-169) + reward tracker reset
// ---------------------------------------------------------------------------
__device__ int env_reset(const Dev& d, Lane& c) {
    c.t = -1;
    c.deaths = 0;
    c.zd = 0;
    c.n_order = 0;
    // new World: empty things / decoration
    uint4* occ4 = (uint4*)(d.occ + (size_t)c.e * d.occ_stride);
    for (int i = 0; i < d.occ_stride / 16; i++) occ4[i] = make_uint4(0, 0, 0, 0);
    uint32_t* dead = d.dead + (size_t)c.e * d.DW;
    for (int i = 0; i < d.DW; i++) dead[i] = 0;
    for (int s = 0; s < d.E; s++) LPR(c, s) = 0;
    // map obstacles re-enter the dict with their carried-over HP (game.py:154-155)
    int any_nonpos = 0;
    for (int w = 0; w < d.OW; w++) {
        int nb = min(32, d.O - 32 * w);
        d.obst_present[(size_t)c.e * d.OW + w] = nb == 32 ? 0xffffffffu : ((1u << nb) - 1u);
        any_nonpos |= d.obst_nonpos[(size_t)c.e * d.OW + w] != 0;
    }
    c.odirty = any_nonpos;
    // players: Player() picks a random weapon unless its module gives one (things.py:113-116)
    for (int p = 0; p < d.P; p++) {
        int s = d.A + p, w;
        int bt = d.bot_types[p];
        if (bt == ZS_BOT_TERMINATOR) w = ZS_WEAPON_SHOTGUN;     // terminator.py:40-42
        else if (bt == ZS_BOT_SNIPER) w = ZS_WEAPON_RIFLE;      // sniper.py:22-24
        else {                                                  // choice([Gun, Shotgun, Rifle, Knife, Axe])
            int k = rng_below(c.rng, 5);
            w = k == 0 ? ZS_WEAPON_GUN : k == 1 ? ZS_WEAPON_SHOTGUN : k == 2 ? ZS_WEAPON_RIFLE : k == 3 ? ZS_WEAPON_KNIFE : ZS_WEAPON_AXE;
        }
        LW(c, s) = (uint8_t)w;
        LL(c, s) = 100;
    }
    // agents: WeaponFactory.create_player_weapon (weapons.py:28-45)
    for (int a = 0; a < d.A; a++) {
        int w = d.agent_weapons[a];
        if (w == ZS_WEAPON_RANDOM) {  // choice([Knife(), Axe(), Gun(), Rifle(), Shotgun()])
            int k = rng_below(c.rng, 5);
            w = k == 0 ? ZS_WEAPON_KNIFE : k == 1 ? ZS_WEAPON_AXE : k == 2 ? ZS_WEAPON_GUN : k == 3 ? ZS_WEAPON_RIFLE : ZS_WEAPON_SHOTGUN;
        }
        LW(c, a) = (uint8_t)w;
        LL(c, a) = 100;
    }
    for (int p = 0; p < d.P; p++) LM(c, p) = (uint8_t)(d.A + p);
    int rc = spawn_in_random(d, c, d.P, d.pspawn, d.nps, 1);
    if (rc) return rc;
    for (int a = 0; a < d.A; a++) LM(c, a) = (uint8_t)a;
    rc = spawn_in_random(d, c, d.A, d.pspawn, d.nps, 1);
    if (rc) return rc;
    spawn_zombies(d, c, d.initial_zombies);
    c.prevzd = 0;
    for (int a = 0; a < d.A; a++) {
        d.prev_life[(size_t)a * d.N + c.e] = LL(c, a);
        d.listed[(size_t)a * d.N + c.e] = 1;
    }
    c.epsteps = 0;
    return ZS_OK;
}

// ---------------------------------------------------------------------------
// decisions (start-of-tick state)
// ---------------------------------------------------------------------------
// Zombie.next_step (things.py:70-105)
__device__ void decide_zombie(const Dev& d, Lane& c, int s, int& kind, int& tgt) {
    int p = LP(c, s), x = unpack_x(p), y = unpack_y(p);
    int freemask = 0;
    for (int k = 0; k < 4; k++)  // possible_moves: not in things, not bounds-checked (utils.py:47-52)
        if (thing_at(d, c, x + c_adj_dx[k], y + c_adj_dy[k]) == NOTHING) freemask |= 1 << k;
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
        // blocked: first Box/Wall in sort_by_distance(target, adjacent_positions(self))
        int dd[4];
        for (int k = 0; k < 4; k++) dd[k] = d2(hx, hy, x + c_adj_dx[k], y + c_adj_dy[k]);
        int used = 0;
        for (int r = 0; r < 4; r++) {
            int bk = -1;
            for (int k = 0; k < 4; k++)
                if (!((used >> k) & 1) && (bk < 0 || dd[k] < dd[bk])) bk = k;
            used |= 1 << bk;
            int th = thing_at(d, c, x + c_adj_dx[bk], y + c_adj_dy[bk]);
            if (th != NOTHING && th < 0) {
                kind = K_ATTACK;
                tgt = th;
                return;
            }
        }
        kind = K_NONE;
        return;
    }
    if (freemask) {  // wander: random.choice(positions)
        int j = rng_below(c.rng, __popc(freemask));
        int k = 0;
        for (; k < 4; k++)
            if ((freemask >> k) & 1) {
                if (j == 0) break;
                j--;
            }
        kind = K_MOVE;
        tgt = pack_xy(x + c_adj_dx[k], y + c_adj_dy[k]);
        return;
    }
    kind = K_NONE;
}

__device__ __forceinline__ int clamp16(int v) { return v < -16384 ? -16384 : (v > 16383 ? 16383 : v); }

// Agent.next_step (players/agent.py:28-96) on the action triple
__device__ void decide_agent(const Dev& d, Lane& c, int s, const int32_t* act, int& kind, int& tgt) {
    int p = LP(c, s), x = unpack_x(p), y = unpack_y(p);
    int ak = act[0], dx = clamp16(act[1]), dy = clamp16(act[2]);
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
            // Player (agents, bots), Box or Wall; never a Zombie
            if (th != NOTHING && (th < 0 || th < d.A + d.P)) {
                kind = K_HEAL;
                tgt = th;
            }
        }
    } else if (ak == ZS_ACT_HEAL_CLOSEST) {
        int q = closest_in(d, c, x, y, 0, d.A + d.P, s);
        kind = K_HEAL;
        tgt = q >= 0 ? q : s;
    }
}

// scripted bots (players/{terminator,sniper,troll,hamster,randoman}.py)
__device__ void decide_bot(const Dev& d, Lane& c, int s, int& kind, int& tgt) {
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
            if (thing_at(d, c, x + c_adj_dx[k], y + c_adj_dy[k]) == NOTHING) freemask |= 1 << k;
        if (freemask) {
            int j = rng_below(c.rng, __popc(freemask));
            int k = 0;
            for (; k < 4; k++)
                if ((freemask >> k) & 1) {
                    if (j == 0) break;
                    j--;
                }
            kind = K_MOVE;
            tgt = pack_xy(x + c_adj_dx[k], y + c_adj_dy[k]);
        }
    } else if (bt == ZS_BOT_RANDOMAN) {  // randoman.py:9-21
        int a = rng_below(c.rng, 3);       // choice(('move', 'attack', 'heal'))
        if (a != 0) {
            // choice(list(things.values())): present obstacles (map order), then dynamic things
            const uint32_t* pres = d.obst_present + (size_t)c.e * d.OW;
            int npo = 0;
            for (int w = 0; w < d.OW; w++) npo += __popc(pres[w]);
            int k = rng_below(c.rng, npo + c.n_order);
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
            int axis = rng_below(c.rng, 2);               // target[choice((0, 1))]
            int delta = rng_below(c.rng, 2) ? 1 : -1;     //   += choice((-1, 1))
            kind = K_MOVE;
            tgt = axis == 0 ? pack_xy(x + delta, y) : pack_xy(x, y + delta);
        }
    }
}

// ---------------------------------------------------------------------------
// rules (rules/{extermination,survival,safehouse,evacuation}.py)
// ---------------------------------------------------------------------------
__device__ void rules_check(const Dev& d, const Lane& c, int& ended, int& won) {
    int pa = 0;  // Rules.players_alive (rules.py:6-11)
    for (int s = 0; s < d.A + d.P; s++) pa |= LL(c, s) > 0;
    if (d.rules == ZS_RULES_EXTERMINATION) {
        int za = 0;
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
    } else {  // evacuation
        int total = d.A + d.P;
        unsigned long long alive = 0;
        int na = 0;
        // get_all_players order = players then agents; the component test is order-free
        for (int s = 0; s < total; s++)
            if (LL(c, s) > 0) {
                alive |= 1ull << s;
                na++;
            }
        int half = 2 * na >= total;
        if (half) {
            // flood fill from alive_players[0] (the first alive bot, else the first alive agent)
            int first = -1;
            for (int s = d.A; s < total && first < 0; s++)
                if ((alive >> s) & 1ull) first = s;
            for (int s = 0; s < d.A && first < 0; s++)
                if ((alive >> s) & 1ull) first = s;
            unsigned long long together = 0, frontier = 0;
            if (first >= 0) {
                together = frontier = 1ull << first;
            }
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
// one tick of one env (gym_env.py:99-145 / gym/multiagent_env.py:111-171)
// ---------------------------------------------------------------------------
__device__ void env_step(const Dev& d, Lane& c, const int32_t* actions, double* rew, uint8_t* done_out,
                         uint8_t* trunc_out, uint8_t* listed_out) {
    const int A = d.A, E = d.E, N = d.N;
    c.t += 1;
    // dict-order ranks for closest() tie-breaks
    for (int k = 0; k < c.n_order; k++) LR(c, LO(c, k)) = (uint8_t)k;
    // World.get_actions (core.py:80-101): actors in dict order
    int nact = 0;
    for (int k = 0; k < c.n_order; k++) {
        int s = LO(c, k), kind = K_NONE, tgt = 0;
        if (s < A) decide_agent(d, c, s, actions + ((size_t)c.e * A + s) * 3, kind, tgt);
        else if (s < A + d.P) decide_bot(d, c, s, kind, tgt);
        else decide_zombie(d, c, s, kind, tgt);
        LK(c, s) = (uint8_t)kind;
        LT(c, s) = tgt;
        if (kind != K_NONE) LPE(c, nact++) = (uint8_t)s;
    }
    // random.shuffle(actions) (core.py:76)
    for (int i = nact - 1; i >= 1; i--) {
        int j = rng_below(c.rng, i + 1);
        uint8_t tmp = LPE(c, i);
        LPE(c, i) = LPE(c, j);
        LPE(c, j) = tmp;
    }
    // execute_actions (core.py:103-119)
    int nmoved = 0;
    uint8_t* occ = d.occ + (size_t)c.e * d.occ_stride;
    for (int i = 0; i < nact; i++) {
        int s = LPE(c, i), kind = LK(c, s), tgt = LT(c, s);
        int p = LP(c, s), x = unpack_x(p), y = unpack_y(p);
        if (kind == K_MOVE) {  // thing_move (core.py:140-166)
            int tx = unpack_x(tgt), ty = unpack_y(tgt);
            if (in_bounds(d, tx, ty) && thing_at(d, c, tx, ty) == NOTHING && d2(x, y, tx, ty) <= 1) {
                occ[y * d.W + x] = 0;
                occ[ty * d.W + tx] = (uint8_t)(s + 1);
                LP(c, s) = tgt;
                LM(c, nmoved++) = (uint8_t)s;
                LR(c, s) = 255;  // re-inserted at the end of the dict
            }
        } else if (kind == K_ATTACK) {  // thing_attack (core.py:168-184)
            int tp = target_pos(d, c, tgt);
            int w = LW(c, s);
            if (d2(x, y, unpack_x(tp), unpack_y(tp)) <= weapon_r2(w)) {
                int dmg = rng_int(c.rng, weapon_lo(w), weapon_hi(w));
                set_target_life(d, c, tgt, target_life(d, c, tgt) - dmg);
            }
        } else {  // thing_heal (core.py:186-202), HEALING_RANGE = 3
            int tp = target_pos(d, c, tgt);
            if (d2(x, y, unpack_x(tp), unpack_y(tp)) <= 9) {
                int ml = target_maxlife(d, tgt);
                int hl = rng_int(c.rng, ml / 10, ml / 4);
                set_target_life(d, c, tgt, min(ml, target_life(d, c, tgt) + hl));
            }
        }
    }
    {  // dict order after the tick's moves: unmoved in old order, then movers in execution order
        int m = 0;
        for (int k = 0; k < c.n_order; k++) {
            int s = LO(c, k);
            if (LR(c, s) != 255) LO(c, m++) = (uint8_t)s;
        }
        for (int j = 0; j < nmoved; j++) LO(c, m++) = LM(c, j);
    }
    // clean_dead_things (core.py:121-138)
    if (c.odirty) {
        for (int w = 0; w < d.OW; w++) {
            uint32_t* pw = &d.obst_present[(size_t)c.e * d.OW + w];
            uint32_t dead = *pw & d.obst_nonpos[(size_t)c.e * d.OW + w];
            if (dead) {
                *pw &= ~dead;
                c.deaths += __popc(dead);
            }
        }
        c.odirty = 0;
    }
    {
        uint32_t* deadbits = d.dead + (size_t)c.e * d.DW;
        int m = 0;
        for (int k = 0; k < c.n_order; k++) {
            int s = LO(c, k);
            if (LL(c, s) <= 0) {
                int p = LP(c, s), cell = unpack_y(p) * d.W + unpack_x(p);
                deadbits[cell >> 5] |= 1u << (cell & 31);
                occ[cell] = 0;
                LPR(c, s) = 0;
                c.deaths++;
                if (s >= A + d.P) c.zd++;
            } else {
                LO(c, m++) = (uint8_t)s;
            }
        }
        c.n_order = m;
    }
    // reward_tracker.update (gym/reward.py:30-35, 77-86)
    double rs = 0.0;
    if (d.reward_mode == ZS_REWARD_SINGLE) {
        long long sp = 0, sc = 0;
        for (int a = 0; a < A; a++) {
            sp += d.prev_life[(size_t)a * N + c.e];
            sc += LL(c, a);
        }
        double prev = (double)c.prevzd + (double)sp / 100.0;
        double cur = (double)c.zd + (double)sc / 100.0;
        rs = cur - prev;
    } else {
        for (int a = 0; a < A; a++) {
            double prev = (double)c.prevzd + (double)d.prev_life[(size_t)a * N + c.e] / 100.0;
            double cur = (double)c.zd + (double)LL(c, a) / 100.0;
            rew[(size_t)c.e * A + a] = cur - prev;
        }
    }
    for (int a = 0; a < A; a++) d.prev_life[(size_t)a * N + c.e] = LL(c, a);
    c.prevzd = c.zd;
    // spawn_zombies_to_maintain_minimum (game.py:196-201)
    {
        int nz = 0;
        for (int s = A + d.P; s < E; s++) nz += LPR(c, s);
        if (nz < d.minimum_zombies) spawn_zombies(d, c, d.minimum_zombies - nz);
    }
    // rules, end-of-game reward (gym_env.py:130-141, gym/multiagent_env.py:143-162)
    int ended, won, tr = 0;
    rules_check(d, c, ended, won);
    double end_reward = 0.0;
    if (ended) {
        end_reward = won ? 10.0 : -10.0;
    } else {
        int aa = 0;
        for (int a = 0; a < A; a++) aa |= LL(c, a) > 0;
        if (!aa) {
            tr = 1;
            end_reward = -10.0;
        }
    }
    if (d.reward_mode == ZS_REWARD_SINGLE) {
        if (ended || tr) rs += end_reward;
        rew[c.e] = rs;
        for (int a = 0; a < A; a++) {
            if (listed_out) listed_out[(size_t)c.e * A + a] = d.listed[(size_t)a * N + c.e];
        }
    } else {
        for (int a = 0; a < A; a++) {
            uint8_t was = d.listed[(size_t)a * N + c.e];
            if (listed_out) listed_out[(size_t)c.e * A + a] = was;
            double r = rew[(size_t)c.e * A + a];
            if (!was) r = 0.0;
            else if (LL(c, a) > 0) r = r + end_reward;
            rew[(size_t)c.e * A + a] = r;
            d.listed[(size_t)a * N + c.e] = LL(c, a) > 0;
        }
    }
    c.epsteps++;
    if (d.max_steps > 0 && c.epsteps >= d.max_steps) tr = 1;
    done_out[c.e] = (uint8_t)ended;
    trunc_out[c.e] = (uint8_t)tr;
}

// ---------------------------------------------------------------------------
// wave-cooperative MT19937 refill: for every env of the block whose next block
// is not ready, the whole workgroup twists it (3 dependency phases).
// ---------------------------------------------------------------------------
__device__ void coop_refill(const Dev& d, int base, int count, const uint32_t* lst, uint32_t* tw) {
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int i = 0; i < count; i++) {
        uint32_t st = lst[i];
        if ((st >> 11) & 1u) continue;
        uint32_t slot = (st >> 10) & 1u;
        uint32_t* ring = d.ring + (size_t)(base + i) * ZS_RING_WORDS;
        const uint32_t* src = ring + slot * ZS_MT_N;
        uint32_t* dst = ring + (slot ^ 1u) * ZS_MT_N;
        for (int k = tid; k < ZS_MT_N; k += nt) tw[k] = src[k];
        __syncthreads();
        uint32_t* nw = tw + ZS_MT_N;
        for (int k = tid; k < ZS_MT_N - ZS_MT_M; k += nt) nw[k] = mt_f(tw[k], tw[k + 1], tw[k + ZS_MT_M]);
        __syncthreads();
        for (int k = (ZS_MT_N - ZS_MT_M) + tid; k < 2 * (ZS_MT_N - ZS_MT_M); k += nt)
            nw[k] = mt_f(tw[k], tw[k + 1], nw[k + ZS_MT_M - ZS_MT_N]);
        __syncthreads();
        for (int k = 2 * (ZS_MT_N - ZS_MT_M) + tid; k < ZS_MT_N; k += nt)
            nw[k] = mt_f(tw[k], k + 1 < ZS_MT_N ? tw[k + 1] : nw[0], nw[k + ZS_MT_M - ZS_MT_N]);
        __syncthreads();
        for (int k = tid; k < ZS_MT_N; k += nt) dst[k] = nw[k];
        if (tid == 0) d.rngst[base + i] = st | (1u << 11);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// the step / reset kernel: one lane per env, state staged through LDS
// ---------------------------------------------------------------------------
enum { MODE_STEP = 0, MODE_RESET = 1 };

__global__ void __launch_bounds__(64) k_tick(Dev d, int mode, const uint8_t* mask, const int32_t* actions,
                                             double* rew, uint8_t* done_out, uint8_t* trunc_out,
                                             uint8_t* listed_out, uint8_t* reset_out, int* err_out) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int wg = blockDim.x, lane = threadIdx.x, E = d.E, N = d.N;
    const int base = blockIdx.x * wg;
    const int e = base + lane;
    uint32_t* tw = (uint32_t*)smem;                       // 2 x 624 words
    uint32_t* lst = tw + 2 * ZS_MT_N;                     // wg words
    Lane c;
    c.e = e;
    c.lane = lane;
    c.wg = wg;
    uint8_t* p = smem + (2 * ZS_MT_N + wg) * 4;
    c.lpos = (int32_t*)p;
    p += (size_t)E * wg * 4;
    c.llife = (int32_t*)p;
    p += (size_t)E * wg * 4;
    c.ltgt = (int32_t*)p;
    p += (size_t)E * wg * 4;
    c.lweap = p;
    p += (size_t)E * wg;
    c.lpres = p;
    p += (size_t)E * wg;
    c.lorder = p;
    p += (size_t)E * wg;
    c.lrank = p;
    p += (size_t)E * wg;
    c.lkind = p;
    p += (size_t)E * wg;
    c.lperm = p;
    p += (size_t)E * wg;
    c.lmoved = p;

    if (e < N) {
        for (int s = 0; s < E; s++) {
            LP(c, s) = d.pos[(size_t)s * N + e];
            LL(c, s) = d.life[(size_t)s * N + e];
            LW(c, s) = d.weapon[(size_t)s * N + e];
            LPR(c, s) = d.present[(size_t)s * N + e];
            LO(c, s) = d.order[(size_t)s * N + e];
        }
        c.t = d.scal[S_T * N + e];
        c.deaths = d.scal[S_DEATHS * N + e];
        c.zd = d.scal[S_ZD * N + e];
        c.epsteps = d.scal[S_EPSTEPS * N + e];
        c.n_order = d.scal[S_NORDER * N + e];
        c.prevzd = d.scal[S_PREVZD * N + e];
        c.serial = d.scal[S_SERIAL * N + e];
        c.odirty = d.scal[S_ODIRTY * N + e];
        int needs_reset = d.scal[S_NEEDRESET * N + e];
        c.rng.ring = d.ring + (size_t)e * ZS_RING_WORDS;
        c.rng.st = d.rngst[e];

        int do_reset = mode == MODE_RESET ? (mask == nullptr || mask[e]) : needs_reset;
        int did_step = 0;
        if (do_reset) {
            int rc = env_reset(d, c);
            if (rc && err_out) atomicMax(err_out, rc);
            needs_reset = 0;
            if (mode == MODE_STEP) {
                for (int a = 0; a < (d.reward_mode == ZS_REWARD_SINGLE ? 1 : d.A); a++)
                    rew[(size_t)e * (d.reward_mode == ZS_REWARD_SINGLE ? 1 : d.A) + a] = 0.0;
                done_out[e] = 0;
                trunc_out[e] = 0;
                if (listed_out)
                    for (int a = 0; a < d.A; a++) listed_out[(size_t)e * d.A + a] = 1;
            }
        } else if (mode == MODE_STEP) {
            env_step(d, c, actions, rew, done_out, trunc_out, listed_out);
            did_step = 1;
            if ((done_out[e] || trunc_out[e]) && (d.flags & ZS_FLAG_AUTORESET)) needs_reset = 1;
        }
        if (mode == MODE_STEP && reset_out) reset_out[e] = (uint8_t)do_reset;
        (void)did_step;

        for (int s = 0; s < E; s++) {
            d.pos[(size_t)s * N + e] = LP(c, s);
            d.life[(size_t)s * N + e] = LL(c, s);
            d.weapon[(size_t)s * N + e] = LW(c, s);
            d.present[(size_t)s * N + e] = LPR(c, s);
            d.order[(size_t)s * N + e] = LO(c, s);
        }
        d.scal[S_T * N + e] = c.t;
        d.scal[S_DEATHS * N + e] = c.deaths;
        d.scal[S_ZD * N + e] = c.zd;
        d.scal[S_EPSTEPS * N + e] = c.epsteps;
        d.scal[S_NORDER * N + e] = c.n_order;
        d.scal[S_PREVZD * N + e] = c.prevzd;
        d.scal[S_SERIAL * N + e] = c.serial;
        d.scal[S_ODIRTY * N + e] = c.odirty;
        d.scal[S_NEEDRESET * N + e] = needs_reset;
        d.rngst[e] = c.rng.st;
        lst[lane] = c.rng.st;
    }
    __syncthreads();
    coop_refill(d, base, min(wg, N - base), lst, tw);
}

// ---------------------------------------------------------------------------
// observations (gym/observation.py:36-173): one workgroup per env, one thread per cell
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) k_obs(Dev d, T* out, const uint8_t* mask) {
    const int e = blockIdx.x;
    if (mask && !mask[e]) return;
    const bool world = d.obs_scope == ZS_OBS_WORLD;
    const int nobs = world ? 1 : (d.reward_mode == ZS_REWARD_MULTI ? d.A : 1);
    const int hh = world ? d.H : d.obs_w, ww = world ? d.W : d.obs_w, half = d.obs_w / 2;
    const int C = d.obs_enc == ZS_ENC_CHANNELS ? 3 : 1;
    const long plane = (long)hh * ww;
    T* o = out + (size_t)e * nobs * C * plane;
    const uint8_t* occ = d.occ + (size_t)e * d.occ_stride;
    const uint32_t* pres = d.obst_present + (size_t)e * d.OW;
    const uint32_t* deadb = d.dead + (size_t)e * d.DW;
    for (long idx = threadIdx.x; idx < nobs * plane; idx += blockDim.x) {
        int a = (int)(idx / plane);
        int cell = (int)(idx - (long)a * plane);
        int r = cell / ww, q = cell - r * ww;
        int x, y;
        if (world) {
            x = q;
            y = r;
        } else {
            int32_t ap = d.pos[(size_t)a * d.N + e];
            x = unpack_x(ap) - half + q;
            y = unpack_y(ap) - half + r;
        }
        int code, life, weapon = 0;
        if (x < 0 || y < 0 || x >= d.W || y >= d.H) {  // Wall(position) out of bounds
            code = ZS_THING_WALL;
            life = 200;
        } else {
            int mc = y * d.W + x;
            int s = (int)occ[mc] - 1;
            if (s >= 0) {
                life = d.life[(size_t)s * d.N + e];
                weapon = d.weapon[(size_t)s * d.N + e];
                code = s < d.A ? (d.obs_enc == ZS_ENC_CHANNELS ? d.agent_codes[s] : ZS_THING_AGENT)
                               : (s < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
            } else {
                int oi = d.cellmap[mc];
                if (oi >= 0 && ((pres[oi >> 5] >> (oi & 31)) & 1u)) {
                    code = d.obst_kind[oi];
                    life = d.obst_hp[(size_t)e * d.O + oi];
                } else {
                    life = 0;
                    code = ((deadb[mc >> 5] >> (mc & 31)) & 1u)             ? ZS_THING_DEADBODY
                           : ((d.objbits[mc >> 5] >> (mc & 31)) & 1u) ? ZS_THING_OBJECTIVE
                                                                             : ZS_THING_NONE;
                }
            }
        }
        T* oa = o + (size_t)a * C * plane + cell;
        if (C == 1) {
            int64_t adj = life < 100 ? life : 100;
            oa[0] = (T)(256 * (int64_t)code + 16 * (int64_t)weapon + floordiv100(15 * adj));
        } else {
            oa[0] = (T)code;
            oa[plane] = (T)life;
            oa[2 * plane] = (T)weapon;
        }
    }
}

// ---------------------------------------------------------------------------
// seeding: random.seed(int) (init_by_array over abs(n) in 32-bit little-endian words)
// ---------------------------------------------------------------------------
__global__ void k_seed(Dev d, int env0, int n, const uint64_t* seeds) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int e = env0 + i;
    uint64_t sd = seeds[i];
    d.seeds[e] = sd;
    uint32_t* mt = d.ring + (size_t)e * ZS_RING_WORDS;
    uint32_t key[2] = {(uint32_t)sd, (uint32_t)(sd >> 32)};
    int klen = (sd >> 32) ? 2 : 1;
    mt[0] = 19650218u;
    for (int k = 1; k < ZS_MT_N; k++) mt[k] = 1812433253u * (mt[k - 1] ^ (mt[k - 1] >> 30)) + (uint32_t)k;
    int a = 1, b = 0;
    for (int k = (ZS_MT_N > klen ? ZS_MT_N : klen); k; k--) {
        mt[a] = (mt[a] ^ ((mt[a - 1] ^ (mt[a - 1] >> 30)) * 1664525u)) + key[b] + (uint32_t)b;
        a++;
        b++;
        if (a >= ZS_MT_N) {
            mt[0] = mt[ZS_MT_N - 1];
            a = 1;
        }
        if (b >= klen) b = 0;
    }
    for (int k = ZS_MT_N - 1; k; k--) {
        mt[a] = (mt[a] ^ ((mt[a - 1] ^ (mt[a - 1] >> 30)) * 1566083941u)) - (uint32_t)a;
        a++;
        if (a >= ZS_MT_N) {
            mt[0] = mt[ZS_MT_N - 1];
            a = 1;
        }
    }
    mt[0] = 0x80000000u;
    // the seeded state is x[0..623]; the first draw twists, so the output stream starts at x[624]
    mt_twist_serial(mt + ZS_MT_N, mt);  // block 1 -> slot 1 (current)
    mt_twist_serial(mt, mt + ZS_MT_N);  // block 2 -> slot 0 (next, ready)
    d.rngst[e] = 0u | (1u << 10) | (1u << 11);
}

// ---------------------------------------------------------------------------
// bench / parity action stream (libzombsole_amd/actions.py)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__constant__ int32_t c_discrete[7][3] = {{ZS_ACT_MOVE, 0, 1},  {ZS_ACT_MOVE, -1, 0},       {ZS_ACT_MOVE, 0, -1},
                                         {ZS_ACT_MOVE, 1, 0},  {ZS_ACT_ATTACK_CLOSEST, 0, 0}, {ZS_ACT_HEAL, 0, 0},
                                         {ZS_ACT_HEAL_CLOSEST, 0, 0}};

__global__ void k_gen_actions(Dev d, uint64_t step, int n_discrete, int32_t* act) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.N * d.A) return;
    int e = i / d.A, a = i - e * d.A;
    uint64_t h = splitmix64(splitmix64(splitmix64(d.seeds[e]) ^ step) ^ (uint64_t)a);
    int id = (int)(h % (uint64_t)n_discrete);
    act[(size_t)i * 3 + 0] = c_discrete[id][0];
    act[(size_t)i * 3 + 1] = c_discrete[id][1];
    act[(size_t)i * 3 + 2] = c_discrete[id][2];
}

// ---------------------------------------------------------------------------
// state views (one env, one thread; test pokes)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int state_words(const Dev& d) {
    return ZS_STATE_HEADER + ZS_STATE_ENTITY_WORDS * d.E + d.E + 2 * d.O + 2 * d.A + d.DW;
}

__global__ void k_get_state(Dev d, int e, int32_t* buf) {
    if (threadIdx.x != 0) return;
    const int N = d.N, E = d.E;
    int32_t* b = buf;
    b[0] = d.scal[S_T * N + e];
    b[1] = d.scal[S_DEATHS * N + e];
    b[2] = d.scal[S_ZD * N + e];
    b[3] = d.scal[S_EPSTEPS * N + e];
    b[4] = d.scal[S_NORDER * N + e];
    b[5] = d.scal[S_NEEDRESET * N + e];
    b[6] = E;
    b[7] = d.O;
    b[8] = d.W;
    b[9] = d.H;
    b[10] = d.scal[S_PREVZD * N + e];
    int nz = 0;
    for (int s = d.A + d.P; s < E; s++) nz += d.present[(size_t)s * N + e];
    b[11] = nz;
    b[12] = b[13] = b[14] = b[15] = 0;
    int32_t* r = b + ZS_STATE_HEADER;
    for (int s = 0; s < E; s++, r += ZS_STATE_ENTITY_WORDS) {
        int32_t p = d.pos[(size_t)s * N + e];
        r[0] = s < d.A ? ZS_THING_AGENT : (s < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
        r[1] = d.present[(size_t)s * N + e];
        r[2] = unpack_x(p);
        r[3] = unpack_y(p);
        r[4] = d.life[(size_t)s * N + e];
        r[5] = d.weapon[(size_t)s * N + e];
        r[6] = s < d.A ? s : (s < d.A + d.P ? s - d.A : 0);
        r[7] = (int32_t)d.serial[(size_t)s * N + e];
    }
    for (int s = 0; s < E; s++) *r++ = d.order[(size_t)s * N + e];
    for (int o = 0; o < d.O; o++) *r++ = d.obst_hp[(size_t)e * d.O + o];
    for (int o = 0; o < d.O; o++) *r++ = (d.obst_present[(size_t)e * d.OW + (o >> 5)] >> (o & 31)) & 1u;
    for (int a = 0; a < d.A; a++) *r++ = d.prev_life[(size_t)a * N + e];
    for (int a = 0; a < d.A; a++) *r++ = d.listed[(size_t)a * N + e];
    for (int w = 0; w < d.DW; w++) *r++ = (int32_t)d.dead[(size_t)e * d.DW + w];
}

__global__ void k_set_state(Dev d, int e, const int32_t* buf) {
    if (threadIdx.x != 0) return;
    const int N = d.N, E = d.E;
    const int32_t* b = buf;
    uint8_t* occ = d.occ + (size_t)e * d.occ_stride;
    for (int s = 0; s < E; s++) {  // lift the old entities off the occupancy grid
        if (d.present[(size_t)s * N + e]) {
            int32_t p = d.pos[(size_t)s * N + e];
            occ[unpack_y(p) * d.W + unpack_x(p)] = 0;
        }
    }
    d.scal[S_T * N + e] = b[0];
    d.scal[S_DEATHS * N + e] = b[1];
    d.scal[S_ZD * N + e] = b[2];
    d.scal[S_EPSTEPS * N + e] = b[3];
    d.scal[S_NORDER * N + e] = b[4];
    d.scal[S_NEEDRESET * N + e] = b[5];
    d.scal[S_PREVZD * N + e] = b[10];
    const int32_t* r = b + ZS_STATE_HEADER;
    for (int s = 0; s < E; s++, r += ZS_STATE_ENTITY_WORDS) {
        d.present[(size_t)s * N + e] = (uint8_t)r[1];
        d.pos[(size_t)s * N + e] = pack_xy(r[2], r[3]);
        d.life[(size_t)s * N + e] = r[4];
        d.weapon[(size_t)s * N + e] = (uint8_t)r[5];
        d.serial[(size_t)s * N + e] = (uint32_t)r[7];
        if (r[1]) occ[r[3] * d.W + r[2]] = (uint8_t)(s + 1);
    }
    for (int s = 0; s < E; s++) d.order[(size_t)s * N + e] = (uint8_t)*r++;
    int any_nonpos = 0;
    for (int o = 0; o < d.O; o++) {
        int v = *r++;
        d.obst_hp[(size_t)e * d.O + o] = v;
        uint32_t* w = &d.obst_nonpos[(size_t)e * d.OW + (o >> 5)];
        *w = v <= 0 ? (*w | (1u << (o & 31))) : (*w & ~(1u << (o & 31)));
        any_nonpos |= v <= 0;
    }
    for (int o = 0; o < d.O; o++) {
        uint32_t* w = &d.obst_present[(size_t)e * d.OW + (o >> 5)];
        *w = *r++ ? (*w | (1u << (o & 31))) : (*w & ~(1u << (o & 31)));
    }
    d.scal[S_ODIRTY * N + e] = any_nonpos;
    for (int a = 0; a < d.A; a++) d.prev_life[(size_t)a * N + e] = *r++;
    for (int a = 0; a < d.A; a++) d.listed[(size_t)a * N + e] = (uint8_t)*r++;
    for (int w = 0; w < d.DW; w++) d.dead[(size_t)e * d.DW + w] = (uint32_t)*r++;
}

__global__ void k_init_obstacles(Dev d) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)d.N * d.O) return;
    int o = (int)(i % d.O);
    d.obst_hp[i] = d.obst_kind[o] == ZS_THING_BOX ? 10 : 200;  // Box / Wall MAX_LIFE
}

// ===========================================================================
// host side: C ABI
// ===========================================================================
static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t _e = (x);                                                                   \
        if (_e != hipSuccess) return fail(ZS_EHIP, std::string(#x ": ") + hipGetErrorString(_e)); \
    } while (0)

struct zs_handle {
    zs_config cfg;
    int device;
    Dev d;
    int wg;
    size_t lds;
    int state_words;
    std::vector<void*> allocs;
    int32_t* d_state;
    uint64_t* d_seedbuf;
    int* d_err;
    // diagnostics: HIP events bracketing every k_tick / k_obs launch on its stream
    int prof = 0;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, int>> ev_tick, ev_obs;  // (start, end) indices into ev_pool
    size_t ev_next = 0;
};

static hipEvent_t prof_event(zs_handle* h, int* idx) {
    if (h->ev_next == h->ev_pool.size()) {
        hipEvent_t ev;
        if (hipEventCreate(&ev) != hipSuccess) return nullptr;
        h->ev_pool.push_back(ev);
    }
    *idx = (int)h->ev_next;
    return h->ev_pool[h->ev_next++];
}

extern "C" const char* zs_last_error(void) { return g_err.c_str(); }

template <typename T>
static int dalloc(zs_handle* h, T** p, size_t count) {
    size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    hipError_t e = hipMalloc((void**)p, bytes);
    if (e != hipSuccess) return fail(ZS_EHIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    h->allocs.push_back(*p);
    e = hipMemset(*p, 0, bytes);
    if (e != hipSuccess) return fail(ZS_EHIP, std::string("hipMemset: ") + hipGetErrorString(e));
    return ZS_OK;
}

template <typename T>
static int dupload(zs_handle* h, T** p, const std::vector<T>& v) {
    int rc = dalloc(h, p, v.size());
    if (rc) return rc;
    if (!v.empty()) HIPCHK(hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return ZS_OK;
}

static void free_all(zs_handle* h) {
    for (void* p : h->allocs) (void)hipFree(p);
    h->allocs.clear();
    for (hipEvent_t ev : h->ev_pool) (void)hipEventDestroy(ev);
    h->ev_pool.clear();
}

extern "C" int zs_destroy(zs_handle* h) {
    if (!h) return ZS_OK;
    (void)hipSetDevice(h->device);
    free_all(h);
    delete h;
    return ZS_OK;
}

static int validate(const zs_config* c) {
    const zs_map_desc& m = c->map;
    if (!c || c->num_envs < 1) return fail(ZS_EINVAL, "num_envs must be >= 1");
    if (m.width < 1 || m.height < 1 || m.width > 16000 || m.height > 16000 || (long)m.width * m.height > (1L << 24))
        return fail(ZS_EINVAL, "map size out of range");
    if (c->num_agents < 1) return fail(ZS_EINVAL, "at least one agent is required");
    if (c->num_bots < 0 || c->initial_zombies < 0 || c->minimum_zombies < 0) return fail(ZS_EINVAL, "negative count");
    long E = (long)c->num_agents + c->num_bots + std::max(c->initial_zombies, c->minimum_zombies);
    if (E > 254) return fail(ZS_EINVAL, "agents + bots + max(initial, minimum) zombies must be <= 254");
    if (c->rules == ZS_RULES_EVACUATION && c->num_agents + c->num_bots > 64)
        return fail(ZS_EINVAL, "evacuation rules support at most 64 players");
    if (c->rules < 0 || c->rules > 3) return fail(ZS_EINVAL, "bad rules id");
    if (c->obs_scope == ZS_OBS_SURROUNDINGS && (c->obs_width <= 1 || c->obs_width % 2 == 0))
        return fail(ZS_EINVAL, "surroundings width must be an odd number greater than 1");
    if (c->obs_dtype < 0 || c->obs_dtype > 2) return fail(ZS_EINVAL, "bad obs dtype");
    for (int i = 0; i < m.n_obstacles; i++) {
        int x = m.obstacle_xy[2 * i], y = m.obstacle_xy[2 * i + 1];
        if (x < 0 || y < 0 || x >= m.width || y >= m.height) return fail(ZS_EINVAL, "obstacle out of bounds");
        if (m.obstacle_kind[i] != ZS_THING_BOX && m.obstacle_kind[i] != ZS_THING_WALL) return fail(ZS_EINVAL, "bad obstacle kind");
    }
    const int32_t* lists[3] = {m.objective_xy, m.player_spawn_xy, m.zombie_spawn_xy};
    int ns[3] = {m.n_objectives, m.n_player_spawns, m.n_zombie_spawns};
    for (int l = 0; l < 3; l++)
        for (int i = 0; i < ns[l]; i++) {
            int x = lists[l][2 * i], y = lists[l][2 * i + 1];
            if (x < 0 || y < 0 || x >= m.width || y >= m.height) return fail(ZS_EINVAL, "map list entry out of bounds");
        }
    for (int a = 0; a < c->num_agents; a++) {
        int w = c->agent_weapons[a];
        if (!(w == ZS_WEAPON_KNIFE || w == ZS_WEAPON_AXE || w == ZS_WEAPON_GUN || w == ZS_WEAPON_RIFLE ||
              w == ZS_WEAPON_SHOTGUN || w == ZS_WEAPON_RANDOM))
            return fail(ZS_EINVAL, "bad agent weapon");
    }
    for (int p = 0; p < c->num_bots; p++)
        if (c->bot_types[p] < ZS_BOT_TERMINATOR || c->bot_types[p] > ZS_BOT_RANDOMAN) return fail(ZS_EINVAL, "bad bot type");
    return ZS_OK;
}

static size_t lds_for(int wg, int E) { return (size_t)(2 * ZS_MT_N + wg) * 4 + (size_t)wg * E * (3 * 4 + 7); }

extern "C" int zs_create(const zs_config* cfg, int device, zs_handle** out) {
    if (!cfg || !out) return fail(ZS_EINVAL, "null argument");
    int rc = validate(cfg);
    if (rc) return rc;
    HIPCHK(hipSetDevice(device));
    zs_handle* h = new zs_handle();
    h->cfg = *cfg;
    h->device = device;
    const zs_map_desc& m = cfg->map;
    Dev& d = h->d;
    memset(&d, 0, sizeof(d));
    d.N = cfg->num_envs;
    d.W = m.width;
    d.H = m.height;
    d.O = m.n_obstacles;
    d.A = cfg->num_agents;
    d.P = cfg->num_bots;
    d.Z = std::max(cfg->initial_zombies, cfg->minimum_zombies);
    d.E = d.A + d.P + d.Z;
    d.OW = (d.O + 31) / 32;
    d.DW = (d.W * d.H + 31) / 32;
    d.nps = m.n_player_spawns;
    d.nzs = m.n_zombie_spawns;
    d.nobj = m.n_objectives;
    d.ncand = std::max(d.nps ? d.nps : d.W * d.H, d.nzs ? d.nzs : d.W * d.H);
    d.occ_stride = ((d.W * d.H + 15) / 16) * 16;
    d.rules = cfg->rules;
    d.reward_mode = cfg->reward_mode;
    d.obs_scope = cfg->obs_scope;
    d.obs_enc = cfg->obs_encoding;
    d.obs_w = cfg->obs_width;
    d.obs_dtype = cfg->obs_dtype;
    d.max_steps = cfg->max_episode_steps;
    d.initial_zombies = cfg->initial_zombies;
    d.minimum_zombies = cfg->minimum_zombies;
    d.flags = cfg->flags;

    // static tables
    std::vector<int16_t> cellmap((size_t)d.W * d.H, -1);
    std::vector<int32_t> oxy(d.O);
    std::vector<uint8_t> okind(d.O);
    for (int i = 0; i < d.O; i++) {
        int x = m.obstacle_xy[2 * i], y = m.obstacle_xy[2 * i + 1];
        if (cellmap[(size_t)y * d.W + x] != -1) {
            delete h;
            return fail(ZS_EINVAL, "two obstacles on one cell");
        }
        cellmap[(size_t)y * d.W + x] = (int16_t)i;
        oxy[i] = (int32_t)((uint32_t)x | ((uint32_t)y << 16));
        okind[i] = m.obstacle_kind[i];
    }
    if (d.O > 32767) {
        delete h;
        return fail(ZS_EINVAL, "too many obstacles");
    }
    std::vector<uint32_t> objbits(d.DW, 0);
    for (int i = 0; i < m.n_objectives; i++) {
        int cell = m.objective_xy[2 * i + 1] * d.W + m.objective_xy[2 * i];
        objbits[cell >> 5] |= 1u << (cell & 31);
    }
    auto packlist = [](const int32_t* xy, int n) {
        std::vector<int32_t> v(n);
        for (int i = 0; i < n; i++) v[i] = (int32_t)((uint32_t)xy[2 * i] | ((uint32_t)xy[2 * i + 1] << 16));
        return v;
    };
    std::vector<int32_t> ps = packlist(m.player_spawn_xy, d.nps), zs = packlist(m.zombie_spawn_xy, d.nzs);
    std::vector<int32_t> aw(cfg->agent_weapons, cfg->agent_weapons + d.A);
    std::vector<int32_t> ac(cfg->agent_codes, cfg->agent_codes + d.A);
    std::vector<int32_t> bt(cfg->bot_types, cfg->bot_types + d.P);

#define TRY(x)             \
    do {                   \
        int _r = (x);      \
        if (_r) {          \
            free_all(h);   \
            delete h;      \
            return _r;     \
        }                  \
    } while (0)
    int16_t* p_cellmap;
    uint32_t* p_objbits;
    int32_t *p_oxy, *p_ps, *p_zs, *p_aw, *p_ac, *p_bt;
    uint8_t* p_okind;
    TRY(dupload(h, &p_cellmap, cellmap));
    TRY(dupload(h, &p_objbits, objbits));
    TRY(dupload(h, &p_oxy, oxy));
    TRY(dupload(h, &p_okind, okind));
    TRY(dupload(h, &p_ps, ps));
    TRY(dupload(h, &p_zs, zs));
    TRY(dupload(h, &p_aw, aw));
    TRY(dupload(h, &p_ac, ac));
    TRY(dupload(h, &p_bt, bt));
    d.cellmap = p_cellmap;
    d.objbits = p_objbits;
    d.obst_xy = p_oxy;
    d.obst_kind = p_okind;
    d.pspawn = p_ps;
    d.zspawn = p_zs;
    d.agent_weapons = p_aw;
    d.agent_codes = p_ac;
    d.bot_types = p_bt;
    const size_t N = d.N, E = d.E;
    TRY(dalloc(h, &d.pos, E * N));
    TRY(dalloc(h, &d.life, E * N));
    TRY(dalloc(h, &d.weapon, E * N));
    TRY(dalloc(h, &d.present, E * N));
    TRY(dalloc(h, &d.serial, E * N));
    TRY(dalloc(h, &d.order, E * N));
    TRY(dalloc(h, &d.scal, (size_t)S_NSCAL * N));
    TRY(dalloc(h, &d.prev_life, (size_t)d.A * N));
    TRY(dalloc(h, &d.listed, (size_t)d.A * N));
    TRY(dalloc(h, &d.obst_hp, (size_t)d.O * N));
    TRY(dalloc(h, &d.obst_present, (size_t)d.OW * N));
    TRY(dalloc(h, &d.obst_nonpos, (size_t)d.OW * N));
    TRY(dalloc(h, &d.occ, (size_t)d.occ_stride * N));
    TRY(dalloc(h, &d.dead, (size_t)d.DW * N));
    TRY(dalloc(h, &d.ring, (size_t)ZS_RING_WORDS * N));
    TRY(dalloc(h, &d.rngst, N));
    TRY(dalloc(h, &d.seeds, N));
    TRY(dalloc(h, &d.cand, (size_t)d.ncand * N));
    h->state_words = ZS_STATE_HEADER + ZS_STATE_ENTITY_WORDS * d.E + d.E + 2 * d.O + 2 * d.A + d.DW;
    TRY(dalloc(h, &h->d_state, (size_t)h->state_words));
    TRY(dalloc(h, &h->d_seedbuf, N));
    TRY(dalloc(h, &h->d_err, 1));
    // workgroup: 64 envs (one wave) unless the LDS image of the entity table is too large
    h->wg = 64;
    while (h->wg > 1 && lds_for(h->wg, d.E) > 64 * 1024) h->wg /= 2;
    h->lds = lds_for(h->wg, d.E);
    if (d.O > 0) {
        size_t n = N * d.O;
        hipLaunchKernelGGL(k_init_obstacles, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d);
        hipError_t le = hipGetLastError();
        if (le != hipSuccess) {
            free_all(h);
            delete h;
            return fail(ZS_EHIP, std::string("k_init_obstacles: ") + hipGetErrorString(le));
        }
    }
    // default seeds: env index (every env has a valid stream even if never seeded)
    std::vector<uint64_t> seeds(N);
    for (size_t i = 0; i < N; i++) seeds[i] = i;
    *out = h;
    rc = zs_seed(h, 0, (int)N, seeds.data(), nullptr);
    if (rc) {
        zs_destroy(h);
        *out = nullptr;
        return rc;
    }
    hipError_t se = hipDeviceSynchronize();
    if (se != hipSuccess) {
        zs_destroy(h);
        *out = nullptr;
        return fail(ZS_EHIP, std::string("zs_create sync: ") + hipGetErrorString(se));
    }
    return ZS_OK;
#undef TRY
}

extern "C" int zs_obs_shape(const zs_handle* h, int32_t out[4]) {
    if (!h || !out) return fail(ZS_EINVAL, "null argument");
    const Dev& d = h->d;
    bool world = d.obs_scope == ZS_OBS_WORLD;
    out[0] = world ? 1 : (d.reward_mode == ZS_REWARD_MULTI ? d.A : 1);
    out[1] = d.obs_enc == ZS_ENC_CHANNELS ? 3 : 1;
    out[2] = world ? d.H : d.obs_w;
    out[3] = world ? d.W : d.obs_w;
    return ZS_OK;
}

extern "C" int zs_seed(zs_handle* h, int32_t env0, int32_t n, const uint64_t* seeds_host, void* stream) {
    if (!h || !seeds_host) return fail(ZS_EINVAL, "null argument");
    if (env0 < 0 || n < 0 || env0 + n > h->d.N) return fail(ZS_EINVAL, "env range out of bounds");
    if (n == 0) return ZS_OK;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMemcpyAsync(h->d_seedbuf, seeds_host, sizeof(uint64_t) * n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_seed, dim3((n + 63) / 64), dim3(64), 0, s, h->d, env0, n, h->d_seedbuf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));  // seeds_host may be freed by the caller on return
    return ZS_OK;
}

static int launch_obs(zs_handle* h, void* obs, const uint8_t* mask, hipStream_t s) {
    const Dev& d = h->d;
    if (!obs) return ZS_OK;
    int i0 = -1, i1 = -1;
    if (h->prof) HIPCHK(hipEventRecord(prof_event(h, &i0), s));
    if (d.obs_dtype == ZS_DTYPE_I64)
        hipLaunchKernelGGL(k_obs<int64_t>, dim3(d.N), dim3(256), 0, s, d, (int64_t*)obs, mask);
    else if (d.obs_dtype == ZS_DTYPE_I32)
        hipLaunchKernelGGL(k_obs<int32_t>, dim3(d.N), dim3(256), 0, s, d, (int32_t*)obs, mask);
    else
        hipLaunchKernelGGL(k_obs<int16_t>, dim3(d.N), dim3(256), 0, s, d, (int16_t*)obs, mask);
    HIPCHK(hipGetLastError());
    if (h->prof) {
        HIPCHK(hipEventRecord(prof_event(h, &i1), s));
        h->ev_obs.push_back({i0, i1});
    }
    return ZS_OK;
}

static int launch_tick(zs_handle* h, int mode, const uint8_t* mask, const int32_t* actions, double* rew,
                       uint8_t* done, uint8_t* trunc, uint8_t* listed, uint8_t* reset_out, hipStream_t s) {
    const Dev& d = h->d;
    unsigned grid = (unsigned)((d.N + h->wg - 1) / h->wg);
    int i0 = -1, i1 = -1;
    if (h->prof) HIPCHK(hipEventRecord(prof_event(h, &i0), s));
    hipLaunchKernelGGL(k_tick, dim3(grid), dim3(h->wg), h->lds, s, d, mode, mask, actions, rew, done, trunc, listed,
                       reset_out, h->d_err);
    HIPCHK(hipGetLastError());
    if (h->prof) {
        HIPCHK(hipEventRecord(prof_event(h, &i1), s));
        h->ev_tick.push_back({i0, i1});
    }
    return ZS_OK;
}

extern "C" int zs_reset(zs_handle* h, const uint8_t* env_mask_dev, void* obs_dev, void* stream) {
    if (!h) return fail(ZS_EINVAL, "null handle");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMemsetAsync(h->d_err, 0, sizeof(int), s));
    int rc = launch_tick(h, MODE_RESET, env_mask_dev, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, s);
    if (rc) return rc;
    rc = launch_obs(h, obs_dev, env_mask_dev, s);
    if (rc) return rc;
    int err = 0;
    HIPCHK(hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (err == ZS_ENOSPACE) return fail(ZS_ENOSPACE, "Not enough space to spawn players/agents");
    if (err) return fail(err, "reset failed");
    return ZS_OK;
}

extern "C" int zs_step(zs_handle* h, const int32_t* actions_dev, void* obs_dev, double* rewards_dev, uint8_t* done_dev,
                       uint8_t* trunc_dev, uint8_t* listed_dev, uint8_t* reset_dev, void* stream) {
    if (!h || !actions_dev || !rewards_dev || !done_dev || !trunc_dev) return fail(ZS_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    int rc = launch_tick(h, MODE_STEP, nullptr, actions_dev, rewards_dev, done_dev, trunc_dev, listed_dev, reset_dev, s);
    if (rc) return rc;
    return launch_obs(h, obs_dev, nullptr, s);
}

extern "C" int zs_gen_actions(zs_handle* h, uint64_t step, int32_t n_discrete, int32_t* actions_dev, void* stream) {
    if (!h || !actions_dev) return fail(ZS_EINVAL, "null argument");
    if (n_discrete < 1 || n_discrete > 7) return fail(ZS_EINVAL, "n_discrete must be in 1..7");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    int n = h->d.N * h->d.A;
    hipLaunchKernelGGL(k_gen_actions, dim3((n + 255) / 256), dim3(256), 0, s, h->d, step, n_discrete, actions_dev);
    HIPCHK(hipGetLastError());
    return ZS_OK;
}

extern "C" int zs_state_size(const zs_handle* h, int32_t* n_words) {
    if (!h || !n_words) return fail(ZS_EINVAL, "null argument");
    *n_words = h->state_words;
    return ZS_OK;
}

extern "C" int zs_get_state(zs_handle* h, int32_t env, int32_t* buf_host, void* stream) {
    if (!h || !buf_host) return fail(ZS_EINVAL, "null argument");
    if (env < 0 || env >= h->d.N) return fail(ZS_EINVAL, "env index out of range");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    hipLaunchKernelGGL(k_get_state, dim3(1), dim3(64), 0, s, h->d, env, h->d_state);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(buf_host, h->d_state, sizeof(int32_t) * h->state_words, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return ZS_OK;
}

extern "C" int zs_set_state(zs_handle* h, int32_t env, const int32_t* buf_host, void* stream) {
    if (!h || !buf_host) return fail(ZS_EINVAL, "null argument");
    if (env < 0 || env >= h->d.N) return fail(ZS_EINVAL, "env index out of range");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMemcpyAsync(h->d_state, buf_host, sizeof(int32_t) * h->state_words, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_set_state, dim3(1), dim3(64), 0, s, h->d, env, h->d_state);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    return ZS_OK;
}

// ---------------------------------------------------------------------------
// diagnostics: per-kernel device time from HIP events recorded on the launch stream
// ---------------------------------------------------------------------------
extern "C" int zs_profile(zs_handle* h, int32_t enable) {
    if (!h) return fail(ZS_EINVAL, "null handle");
    h->prof = enable ? 1 : 0;
    h->ev_tick.clear();
    h->ev_obs.clear();
    h->ev_next = 0;
    return ZS_OK;
}

extern "C" int zs_profile_read(zs_handle* h, double* out) {
    if (!h || !out) return fail(ZS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(h->device));
    double tot[2] = {0.0, 0.0};
    std::vector<std::pair<int, int>>* lists[2] = {&h->ev_tick, &h->ev_obs};
    for (int k = 0; k < 2; k++)
        for (auto& pr : *lists[k]) {
            HIPCHK(hipEventSynchronize(h->ev_pool[pr.second]));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, h->ev_pool[pr.first], h->ev_pool[pr.second]));
            tot[k] += ms;
        }
    out[0] = tot[0];
    out[1] = (double)h->ev_tick.size();
    out[2] = tot[1];
    out[3] = (double)h->ev_obs.size();
    h->ev_tick.clear();
    h->ev_obs.clear();
    h->ev_next = 0;
    return ZS_OK;
}
