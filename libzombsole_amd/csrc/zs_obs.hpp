// zs_obs.hpp — the observation encoder (gym/observation.py:36-173), one wave per env.
//
// Observations are the bulk of the bytes a step moves (21 KB per env-step at C3, int64), so the
// encoder is shaped as a store stream with as little per-cell work as possible:
//   * one wave owns one env and writes its whole [nobs][C][h][w] block, so every store
//     instruction of the wave covers 64 consecutive cells of one plane (512 B of int64);
//   * the env's dynamic state is staged once into a wave-private LDS image: a "window map"
//     (one byte per observed cell: entity slot + 1, scattered from the <= E entity positions —
//     the reference's `things` lookup, observation.py:57-66, without a per-cell search), the
//     entities' positions, (code, weapon, present) and life, the dead-body bitmap, obstacle
//     presence and (when it fits) obstacle HP;
//   * the static map (obstacle index and kind, objective flag) is one int32 per cell shared by
//     all envs and served from L1/L2.
// The same two steps (obs_build, obs_stream) run in three places: k_obs (zs_reset, zs_observe,
// and steps whose image does not fit the step launch), the step launch's tick workgroups right
// after an env's tick, and its reset work right after an env's rebuild — so a step writes its
// observations while other workgroups of the same launch are still ticking.
// Per cell: out of bounds -> Wall(200) (observation.py:69-76); entity (things first); present
// obstacle (Box / Wall with its HP); dead body; objective; empty.
#pragma once
#include "zs_device.hpp"

// static per-cell word: bits 0..15 obstacle index + 1 (0 = none), 16..18 obstacle code, bit 20 objective
#define SC_OBST_MASK 0xffffu
#define SC_KIND_SHIFT 16
#define SC_OBJ_BIT (1u << 20)

typedef unsigned int zs_v4u __attribute__((ext_vector_type(4)));
typedef unsigned int zs_v2u __attribute__((ext_vector_type(2)));
typedef int zs_v2i __attribute__((ext_vector_type(2)));
typedef int zs_v4i __attribute__((ext_vector_type(4)));

// observations per env
__host__ __device__ inline int obs_count(int scope, int reward_mode, int A) {
    return scope == ZS_OBS_WORLD ? 1 : (reward_mode == ZS_REWARD_MULTI ? A : 1);
}

// workgroup b of nb -> XCD-contiguous virtual workgroup id (a bijection on [0, nb)).  The hardware
// deals workgroups round-robin to the 8 XCDs; this gives each XCD a contiguous range of envs, so
// the env-minor entity rows one XCD's L2 holds are the rows its own waves read.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x * q + (x < r ? x : r) + k;
}

// Units (envs, or env pairs) of a persistent store-stream kernel dealt so that the chip writes a
// narrow address range at a time: XCD x (workgroups b = x mod 8) owns a contiguous region of the
// units, in proportion to its workgroups; round k of the XCD's gx workgroups covers gx * W consecutive
// units of it, W consecutive ones per workgroup (one per writer wave).  Measured with
// tools/probe/storeceil.hip: whole 21 168-B blocks per wave, consecutive waves of an XCD on consecutive
// blocks ("xcd waveenv") 5.78 TB/s; one block per wave strided over the chip ("chunk 21168") 5.06.
#ifndef ZS_RING_DEAL
#define ZS_RING_DEAL 1
#endif
struct XcdDeal {
    int base, span, off, w, ucount;
    __device__ XcdDeal(int b, int nb, int n_units, int W) : w(W) {
        const int q = nb >> 3, r = nb & 7, x = b & 7, j = b >> 3;
        const int gs = x * q + (x < r ? x : r), gx = q + (x < r);  // XCD x: workgroups [gs, gs + gx)
        const int r0 = (int)((long long)n_units * gs / nb), r1 = (int)((long long)n_units * (gs + gx) / nb);
        base = r0;
        span = gx * W;
        off = j * W;
        const int m = r1 - r0 - off;
        ucount = m <= 0 ? 0 : (m / span) * W + min(m % span, W);
    }
    __device__ int unit(int u) const { return base + (u / w) * span + off + u % w; }
};

__device__ __forceinline__ int floordiv100_i32(int a) {  // Python a // 100
    int q = a / 100;
    if (q * 100 != a && a < 0) q -= 1;
    return q;
}

// A value into an observation element of type T.  Every value fits int32; only an obstacle's
// carried-over life (and the simple code of such a cell) can leave the int16 range, and the int16
// form saturates it (the tick raised ZS_OVF_INT16 when the life got there: zs_overflow).
template <typename T>
__device__ __forceinline__ T obs_val(int64_t v) {
    if constexpr (sizeof(T) == 2) return (T)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
    return (T)v;
}
template <typename T>
__device__ __forceinline__ T obs_val(int v) {
    if constexpr (sizeof(T) == 2) return (T)max(-32768, min(v, 32767));  // v_med3_i32
    return (T)v;
}

// Cache policy of the observation stores (the buffer instructions' aux bits; plain stores: nontemporal).
// int16 blocks (C5) are stored nt (streaming, aux 2): measured on one MI355X (2 runs each), C5's k_obs_ring
// 196 -> 138.5 us and its tick and reset work 9-10 % shorter (the state they read stays cached); int64
// blocks keep the default policy (nt: C3 k_obs_ring 227 -> 302 us, the 8 192-env k_obs_pipe 30.7 -> 57.8).
// -DZS_OBS_AUX=a forces aux a on every dtype (A/B builds).
template <typename T>
__device__ __forceinline__ constexpr int obs_aux() {
#ifdef ZS_OBS_AUX
    return ZS_OBS_AUX;
#else
    return sizeof(T) == 2 ? 2 : 0;
#endif
}
template <typename T>
__device__ __forceinline__ void obs_put(T* p, T v) {
    if constexpr (obs_aux<T>() != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <typename T>
__device__ __forceinline__ void obs_store(T* o, int plane, int cell, bool ch, int code, int life, int weapon) {
    if (!ch) {
        const int adj = life < 100 ? life : 100;
        // 15 * adj // 100 (Python floor division); 32-bit fast path for every reachable life
        const int64_t f = adj >= -(1 << 26) ? (int64_t)floordiv100_i32(15 * adj) : floordiv100(15 * (int64_t)adj);
        obs_put(o + cell, obs_val<T>(256 * (int64_t)code + 16 * (int64_t)weapon + f));
    } else {
        obs_put(o + cell, (T)code);
        obs_put(o + plane + cell, obs_val<T>(life));
        obs_put(o + 2 * plane + cell, (T)weapon);
    }
}

// Fill env e's image (all 64 lanes of the wave).  ent(s, pos, life, weapon, present) reads entity
// slot s from wherever the caller holds it (HBM, or the tick / reset LDS image).
template <typename Ent>
__device__ __forceinline__ void obs_build(const Dev& d, const ObsLayout& L, lu8* img, int e, Ent ent) {
    const int lane = threadIdx.x & 63;
    const int E = d.E, A = d.A;
    const bool world = d.obs_scope == ZS_OBS_WORLD;
    const int nobs = obs_count(d.obs_scope, d.reward_mode, A);
    const int hh = world ? d.H : d.obs_w, ww = world ? d.W : d.obs_w, half = d.obs_w / 2;
    const int plane = hh * ww;
    const bool ch = d.obs_enc == ZS_ENC_CHANNELS;
    li32* pos = (li32*)(img + L.off_pos);
    li32* life = (li32*)(img + L.off_life);
    li32* cw = (li32*)(img + L.off_cw);
    for (int w = lane; w < L.win / 4; w += 64) ((lu32*)img)[w] = 0u;
    for (int s = lane; s < E; s += 64) {
        int p, lf, wp, pr;
        ent(s, p, lf, wp, pr);
        const int code = s < A ? (ch ? d.agent_codes[s] : ZS_THING_AGENT) : (s < A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
        pos[s] = p;
        life[s] = lf;
        cw[s] = code | (wp << 8) | (pr << 16);
    }
    stage_in(d.dead + (size_t)e * d.DW, d.DW, lane, 64, (lu32*)(img + L.off_dead), [](int w) { return w; });
    stage_in(d.obst_present + (size_t)e * d.OW, d.OW, lane, 64, (lu32*)(img + L.off_opres), [](int w) { return w; });
    if (L.hp_cap) stage_in(d.obst_hp + (size_t)e * d.O, d.O, lane, 64, (li32*)(img + L.off_hp), [](int w) { return w; });
    wave_sync();
    if (L.win) {  // scatter the present entities into the window map
        for (int s = lane; s < E; s += 64) {
            if (!((cw[s] >> 16) & 1)) continue;
            const int32_t p = pos[s];
            const int x = unpack_x(p), y = unpack_y(p);
            for (int a = 0; a < nobs; a++) {
                int ox = 0, oy = 0;
                if (!world) {
                    const int32_t ap = pos[a];
                    ox = unpack_x(ap) - half;
                    oy = unpack_y(ap) - half;
                }
                const int dx = x - ox, dy = y - oy;
                if (dx >= 0 && dy >= 0 && dx < ww && dy < hh) img[a * plane + dy * ww + dx] = (uint8_t)(s + 1);
            }
        }
        wave_sync();
    }
}

// static tables (LDS, 4 x DW words): [0, DW) obstacle bits, [DW, 2DW) box bits, [2DW, 3DW)
// objective bits, [3DW, 4DW) obstacles in cells below word w.  With the map's obstacles in
// row-major order (every map-file parse) the obstacle index of a cell is its rank, so these replace
// the per-cell static words and keep the store loop free of global loads: any global load inside
// it would make the wave wait (vmcnt is in order) for every store it has issued before.
__device__ __forceinline__ void obs_stage_static(const Dev& d, lu32* st, int t0, int nt) {
    stage_in(d.obstbits, d.DW, t0, nt, st, [](int w) { return w; });
    stage_in(d.boxbits, d.DW, t0, nt, st + d.DW, [](int w) { return w; });
    stage_in(d.objbits, d.DW, t0, nt, st + 2 * d.DW, [](int w) { return w; });
    stage_in((const uint32_t*)d.oprefix, d.DW, t0, nt, st + 3 * d.DW, [](int w) { return w; });
}

// ---------------------------------------------------------------------------
// Compact image of the store-stream kernels (k_obs_pipe, k_obs_lds), in the same ObsLayout regions:
//   * the entity table is one 8-B pair per slot, {code | weapon << 8 | present << 16, life}, at
//     off_life (the life and code-word regions are adjacent);
//   * obstacle HP is stored with its presence folded in: HP of a present obstacle, ZS_HP_ABSENT for one
//     cleaned up (its cell is then empty, core.py:121-138);
//   * the static tables are interleaved per bitmap word: {obstacle, box, objective bits, obstacles in
//     the cells below the word}, one 16-B read.
// A cell is then five independent LDS reads (window-map byte, static word, dead-body word; then the
// entity pair and the obstacle HP) in two dependency levels and no branch, instead of ten in four.
// ---------------------------------------------------------------------------
#define ZS_HP_ABSENT ((int)0x80000000)
typedef ZS_LDS zs_v4u lv4u;
typedef ZS_LDS zs_v2i lv2i;

__device__ __forceinline__ void obs_stage_static4(const Dev& d, lv4u* st4, int t0, int nt) {
    for (int w = t0; w < d.DW; w += nt)
        st4[w] = zs_v4u{d.obstbits[w], d.boxbits[w], d.objbits[w], (uint32_t)d.oprefix[w]};
}

__device__ __forceinline__ void obs_cell_lds(const Dev& d, const ObsLayout& L, const lv4u* st4, const lu8* img,
                                             const lu8* wm, int cell, int x, int y, int& code, int& lf, int& weapon) {
    const lv2i* ent = (const lv2i*)(img + L.off_life);
    const lu32* dead = (const lu32*)(img + L.off_dead);
    const li32* hpx = (const li32*)(img + L.off_hp);
    const bool inb = (unsigned)x < (unsigned)d.W && (unsigned)y < (unsigned)d.H;
    const int c = inb ? y * d.W + x : 0, w = c >> 5;
    const uint32_t bit = 1u << (c & 31);
    const int sb = wm[cell];  // entity slot + 1, or 0
    const zs_v4u sw = st4[w];
    const uint32_t dw = dead[w];
    const zs_v2i ev = ent[sb ? sb - 1 : 0];
    const bool isob = (sw.x & bit) != 0u;
    const int ohp = hpx[isob ? (int)sw.w + __popc(sw.x & (bit - 1u)) : 0];
    const bool obp = isob && ohp != ZS_HP_ABSENT;
    code = (dw & bit) ? ZS_THING_DEADBODY : (sw.z & bit) ? ZS_THING_OBJECTIVE : ZS_THING_NONE;
    code = obp ? ((sw.y & bit) ? ZS_THING_BOX : ZS_THING_WALL) : code;
    code = sb ? (ev.x & 255) : code;
    code = inb ? code : ZS_THING_WALL;
    lf = sb ? ev.y : (obp ? ohp : 0);
    lf = inb ? lf : 200;
    weapon = (inb && sb) ? ((ev.x >> 8) & 255) : 0;
}

// One agent's 21 x 21 channels block into an LDS staging slot (`ot`, elements of S): this lane's
// cells lane + 64 i.  The lookups of obs_cell_lds are issued level by level for a group of GRP cells
// (window-map byte, static word and dead-body word of every cell of the group; then their entity pairs
// and obstacle HP; then the selects and the slot writes), so the LDS round trips of the group overlap.
// Cell by cell, each cell's slot writes sit between its reads and the next cell's, and (LDS addresses
// the compiler cannot tell apart) every read waits for them: four dependent LDS waits per cell.
#ifndef ZS_OBS_GRP
#define ZS_OBS_GRP 1  // measured on one MI355X (2 runs each): C5 k_obs_lds 241 / 243 us at 1, 286 / 291 at 4
#endif
template <typename S, int GRP = ZS_OBS_GRP>
__device__ __forceinline__ void obs_encode_block(const Dev& d, const ObsLayout& L, const lv4u* st4, const lu8* img,
                                                 const lu8* wm, int ox, int oy, ZS_LDS S* ot, int lane) {
    constexpr int WW = 21, PLANE = WW * WW, PER = (PLANE + 63) / 64;
    const lv2i* ent = (const lv2i*)(img + L.off_life);
    const lu32* dead = (const lu32*)(img + L.off_dead);
    const li32* hpx = (const li32*)(img + L.off_hp);
#pragma unroll
    for (int i0 = 0; i0 < PER; i0 += GRP) {
        constexpr int G2 = GRP;
        int sb[G2];
        zs_v4u sw[G2];
        uint32_t dw[G2], bit[G2];
        bool inb[G2];
#pragma unroll
        for (int k = 0; k < G2; k++) {
            const int i = i0 + k < PER ? i0 + k : PER - 1;
            const int cc = min(lane + 64 * i, PLANE - 1), r = cc / WW, q = cc - r * WW;
            const int x = ox + q, y = oy + r;
            inb[k] = (unsigned)x < (unsigned)d.W && (unsigned)y < (unsigned)d.H;
            const int c = inb[k] ? y * d.W + x : 0;
            bit[k] = 1u << (c & 31);
            sb[k] = wm[cc];
            sw[k] = st4[c >> 5];
            dw[k] = dead[c >> 5];
        }
        zs_v2i ev[G2];
        int ohp[G2];
#pragma unroll
        for (int k = 0; k < G2; k++) {
            ev[k] = ent[sb[k] ? sb[k] - 1 : 0];
            const bool isob = (sw[k].x & bit[k]) != 0u;
            ohp[k] = hpx[isob ? (int)sw[k].w + __popc(sw[k].x & (bit[k] - 1u)) : 0];
        }
#pragma unroll
        for (int k = 0; k < G2; k++) {
            const int cell = lane + 64 * (i0 + k);
            const bool isob = (sw[k].x & bit[k]) != 0u;
            const bool obp = isob && ohp[k] != ZS_HP_ABSENT;
            int code = (dw[k] & bit[k]) ? ZS_THING_DEADBODY : (sw[k].z & bit[k]) ? ZS_THING_OBJECTIVE : ZS_THING_NONE;
            code = obp ? ((sw[k].y & bit[k]) ? ZS_THING_BOX : ZS_THING_WALL) : code;
            code = sb[k] ? (ev[k].x & 255) : code;
            code = inb[k] ? code : ZS_THING_WALL;
            int lf = sb[k] ? ev[k].y : (obp ? ohp[k] : 0);
            lf = inb[k] ? lf : 200;
            const int weapon = (inb[k] && sb[k]) ? ((ev[k].x >> 8) & 255) : 0;
            if (i0 + k < PER && cell < PLANE) {
                ot[cell] = (S)code;
                ot[PLANE + cell] = obs_val<S>(lf);
                ot[2 * PLANE + cell] = (S)weapon;
            }
        }
    }
}

// Stream env e's observations from its image: lane handles cells lane, lane + 64, ... of every
// observation.  out = the base of the [N][nobs][C][h][w] tensor.
//
// Fast path (static tables in st, HP and window map in the image): every lookup is an LDS read and
// the cell's value is selected branch-free.  The registered width (21) is a compile-time constant.
__device__ __forceinline__ void obs_cell_fast(const Dev& d, const ObsLayout& L, const lu32* st, const lu8* img,
                                              const lu8* wm, int cell, int x, int y, int& code, int& lf, int& weapon) {
    const int DW = d.DW, W = d.W, H = d.H;
    const li32* life = (const li32*)(img + L.off_life);
    const li32* cw = (const li32*)(img + L.off_cw);
    const lu32* dead = (const lu32*)(img + L.off_dead);
    const lu32* opres = (const lu32*)(img + L.off_opres);
    const li32* hp = (const li32*)(img + L.off_hp);
    const bool inb = (unsigned)x < (unsigned)W && (unsigned)y < (unsigned)H;
    const int c = inb ? y * W + x : 0, w = c >> 5;
    const uint32_t bit = 1u << (c & 31);
    const int sb = wm[cell];  // entity slot + 1, or 0
    const int sidx = sb ? sb - 1 : 0;
    const int v = cw[sidx], elife = life[sidx];
    const uint32_t ob = st[w], bx = st[DW + w], objw = st[2 * DW + w], dw = dead[w];
    const bool isob = (ob & bit) != 0u;
    const int oi = isob ? (int)st[3 * DW + w] + __popc(ob & (bit - 1u)) : 0;
    const uint32_t opw = opres[oi >> 5];
    const int ohp = hp[oi];
    const bool obp = isob && ((opw >> (oi & 31)) & 1u);
    code = (dw & bit) ? ZS_THING_DEADBODY : (objw & bit) ? ZS_THING_OBJECTIVE : ZS_THING_NONE;
    code = obp ? ((bx & bit) ? ZS_THING_BOX : ZS_THING_WALL) : code;
    code = sb ? (v & 255) : code;
    code = inb ? code : ZS_THING_WALL;
    lf = sb ? elife : (obp ? ohp : 0);
    lf = inb ? lf : 200;
    weapon = (inb && sb) ? ((v >> 8) & 255) : 0;
}

template <typename T, int WW>
__device__ __forceinline__ void obs_stream_fast(const Dev& d, const ObsLayout& L, const lu32* st, const lu8* img, T* out,
                                                int e) {
    const int lane = threadIdx.x & 63;
    const bool world = d.obs_scope == ZS_OBS_WORLD;
    const int nobs = obs_count(d.obs_scope, d.reward_mode, d.A);
    const bool ch = d.obs_enc == ZS_ENC_CHANNELS;
    const li32* pos = (const li32*)(img + L.off_pos);
    if (WW > 0) {  // registered width: compile-time plane and row stepping
        constexpr int PLANE = WW > 0 ? WW * WW : 1, SR = WW > 0 ? 64 / WW : 0, SQ = 64 - SR * WW;
        const int C = ch ? 3 : 1;
        for (int a = 0; a < nobs; a++) {
            const int32_t ap = pos[a];
            const int ox = unpack_x(ap) - WW / 2, oy = unpack_y(ap) - WW / 2;
            const lu8* wm = img + a * PLANE;
            T* o = out + ((size_t)e * nobs + a) * C * PLANE;
            int r = lane / (WW > 0 ? WW : 1), q = lane - r * WW;
            for (int cell = lane; cell < PLANE; cell += 64) {
                int code, lf, weapon;
                obs_cell_fast(d, L, st, img, wm, cell, ox + q, oy + r, code, lf, weapon);
                obs_store(o, PLANE, cell, ch, code, lf, weapon);
                q += SQ;
                r += SR;
                if (q >= WW) {
                    q -= WW;
                    r++;
                }
            }
        }
        return;
    }
    const int W = d.W, H = d.H;
    const int ww = world ? W : d.obs_w, hh = world ? H : d.obs_w, half = ww / 2;
    const int plane = hh * ww, C = ch ? 3 : 1;
    const int step_r = 64 / ww, step_q = 64 - step_r * ww;
    for (int a = 0; a < nobs; a++) {
        int ox = 0, oy = 0;
        if (!world) {
            const int32_t ap = pos[a];
            ox = unpack_x(ap) - half;
            oy = unpack_y(ap) - half;
        }
        T* o = out + ((size_t)e * nobs + a) * C * plane;
        const lu8* wm = img + a * plane;
        int r = lane / ww, q = lane - (lane / ww) * ww;
        for (int cell = lane; cell < plane; cell += 64) {
            int code, lf, weapon;
            obs_cell_fast(d, L, st, img, wm, cell, ox + q, oy + r, code, lf, weapon);
            obs_store(o, plane, cell, ch, code, lf, weapon);
            q += step_q;
            r += step_r;
            if (q >= ww) {
                q -= ww;
                r++;
            }
        }
    }
}

// General path: per-cell static words from L1/L2, HP from HBM when not staged, the per-cell
// entity scan when there is no window map.
template <typename T>
__device__ __forceinline__ void obs_stream_gen(const Dev& d, const ObsLayout& L, const lu8* img, T* out, int e) {
    const int lane = threadIdx.x & 63;
    const int E = d.E;
    const bool world = d.obs_scope == ZS_OBS_WORLD;
    const int nobs = obs_count(d.obs_scope, d.reward_mode, d.A);
    const int hh = world ? d.H : d.obs_w, ww = world ? d.W : d.obs_w, half = d.obs_w / 2;
    const bool ch = d.obs_enc == ZS_ENC_CHANNELS;
    const int plane = hh * ww, C = ch ? 3 : 1;
    const li32* pos = (const li32*)(img + L.off_pos);
    const li32* life = (const li32*)(img + L.off_life);
    const li32* cw = (const li32*)(img + L.off_cw);
    const lu32* dead = (const lu32*)(img + L.off_dead);
    const lu32* opres = (const lu32*)(img + L.off_opres);
    const li32* hp = (const li32*)(img + L.off_hp);
    const int step_r = 64 / ww, step_q = 64 - step_r * ww;
    for (int a = 0; a < nobs; a++) {
        int ox = 0, oy = 0;
        if (!world) {
            const int32_t ap = pos[a];
            ox = unpack_x(ap) - half;
            oy = unpack_y(ap) - half;
        }
        T* o = out + ((size_t)e * nobs + a) * C * plane;
        int r = lane / ww, q = lane - (lane / ww) * ww;
        for (int cell = lane; cell < plane; cell += 64) {
            const int x = ox + q, y = oy + r;
            int code = ZS_THING_WALL, lf = 200, weapon = 0;
            if (x >= 0 && y >= 0 && x < d.W && y < d.H) {
                const int c = y * d.W + x;
                int s = -1;
                if (L.win) {
                    s = (int)img[a * plane + cell] - 1;
                } else {
                    const int32_t pk = pack_xy(x, y);
                    for (int k = 0; k < E && s < 0; k++)
                        if (((cw[k] >> 16) & 1) && pos[k] == pk) s = k;
                }
                if (s >= 0) {
                    const int v = cw[s];
                    code = v & 255;
                    weapon = (v >> 8) & 255;
                    lf = life[s];
                } else {
                    const uint32_t sc = (uint32_t)d.scell[c];
                    const int oi = (int)(sc & SC_OBST_MASK) - 1;
                    lf = 0;
                    if (oi >= 0 && ((opres[oi >> 5] >> (oi & 31)) & 1u)) {
                        code = (int)((sc >> SC_KIND_SHIFT) & 7u);
                        lf = L.hp_cap ? hp[oi] : d.obst_hp[(size_t)e * d.O + oi];
                    } else {
                        code = ((dead[c >> 5] >> (c & 31)) & 1u) ? ZS_THING_DEADBODY
                               : (sc & SC_OBJ_BIT)              ? ZS_THING_OBJECTIVE
                                                                : ZS_THING_NONE;
                    }
                }
            }
            obs_store(o, plane, cell, ch, code, lf, weapon);
            q += step_q;
            r += step_r;
            if (q >= ww) {
                q -= ww;
                r++;
            }
        }
    }
}

// st == nullptr: no static tables staged (maps whose obstacles are not in row-major order)
template <typename T>
__device__ __forceinline__ void obs_stream(const Dev& d, const ObsLayout& L, const lu32* st, const lu8* img, T* out,
                                           int e) {
    if (st && L.hp_cap && L.win && d.O > 0) {
        if (d.obs_scope != ZS_OBS_WORLD && d.obs_w == 21) obs_stream_fast<T, 21>(d, L, st, img, out, e);
        else obs_stream_fast<T, 0>(d, L, st, img, out, e);
    } else {
        obs_stream_gen<T>(d, L, img, out, e);
    }
}

__device__ __forceinline__ void obs_stream_any(const Dev& d, const ObsLayout& L, const lu32* st, const lu8* img,
                                               void* out, int e) {
    if (d.obs_dtype == ZS_DTYPE_I64) obs_stream(d, L, st, img, (int64_t*)out, e);
    else if (d.obs_dtype == ZS_DTYPE_I32) obs_stream(d, L, st, img, (int32_t*)out, e);
    else obs_stream(d, L, st, img, (int16_t*)out, e);
}

// k_obs: blockDim/64 envs per workgroup, one env per wave, wave-private LDS images after the
// workgroup's static tables (stat_words = 4 * DW, or 0).
template <typename T>
__global__ void __launch_bounds__(256) k_obs(Dev d, T* out, const uint8_t* mask, ObsLayout L, int stat_words) {
    if (blockIdx.x == 0 && threadIdx.x == 0) step_tail(d);  // a zs_step's tail (Dev::tail_*)
    extern __shared__ __align__(16) uint8_t smem[];
    const int wave = threadIdx.x >> 6, wpg = blockDim.x >> 6;
    lu32* st = (lu32*)smem;
    if (stat_words) {
        obs_stage_static(d, st, threadIdx.x, blockDim.x);
        __syncthreads();
    }
    const int e = xcd_remap(blockIdx.x, gridDim.x) * wpg + wave;
    if (e >= d.N) return;
    if (mask && !mask[e]) return;
    lu8* img = (lu8*)(smem + stat_words * 4 + wave * L.bytes);
    obs_build(d, L, img, e, [&](int s, int& p, int& lf, int& wp, int& pr) {
        p = d.pos[EIX(d, s, e)];
        lf = d.life[EIX(d, s, e)];
        wp = d.weapon[EIX(d, s, e)];
        pr = d.present[EIX(d, s, e)];
    });
    obs_stream(d, L, stat_words ? st : nullptr, img, out, e);
}

// ---------------------------------------------------------------------------
// k_obs_pipe: the store-stream form of k_obs for the registered shape (surroundings, width 21,
// NOBS observations per env, static tables, staged HP).  A wave stays resident and walks envs
// e0, e0 + waves, ...; the state of its next env is loaded into registers (prefetch) before the
// current env's stores are issued, so the load latency hides under the store stream instead of
// idling the wave slot (a wave that stages and then stores spends ~40 % of its life waiting on the
// staging loads while holding its slot).  The store stream is fully unrolled (NOBS x 7 x C store
// instructions), so the next iteration's wait for the prefetch is an exact vmcnt(#stores) that
// lets the stores stay in flight.
// ---------------------------------------------------------------------------
#ifndef ZS_OBS_PIPE_WAVES
#define ZS_OBS_PIPE_WAVES 4  // register budget: waves per SIMD the compiler must allow
#endif
#define OBS_PF_D 2   // prefetched dead-body words per lane   (DW <= 128: maps up to 4096 cells)
#define OBS_PF_H 8   // prefetched obstacle HP words per lane (O <= 512)

struct ObsPrefetch {
    int32_t pos, life, wp, pr;        // lane s < E: entity slot s
    uint32_t dead[OBS_PF_D];
    uint32_t opres;                   // lane w < OW
    int32_t hp[OBS_PF_H];
    zs_v2u dirty_ahead;               // obs_dirty of the env this prefetch was told to look ahead to
};

// {hp_dirty, dead_dirty} of env e
__device__ __forceinline__ zs_v2u obs_dirty(const Dev& d, int e) { return zs_v2u{d.hp_dirty[e], d.dead_dirty[e]}; }
// dirty masks that read every chunk from the env's own rows: for a kernel's first env, whose masks
// would otherwise be one more load round ahead of its first store (the rows hold the values either way)
#define OBS_OWN_ROWS (zs_v2u{~0u, ~0u})

// Every load is unconditional (addresses clamped into the row): a load under a lane predicate
// becomes a branch whose join needs the loaded value, i.e. a wait right after the prefetch.
// dirty = obs_dirty(d, e), loaded by an earlier prefetch (its `ahead` env): an obstacle of a clean HP
// chunk reads hp_init instead of the env's row, a clean dead-body chunk reads dead_zero, and the address
// selects wait on nothing in flight.
__device__ __forceinline__ void obs_prefetch_env(const Dev& d, int e, zs_v2u dirty, ObsPrefetch& f) {
    const int lane = threadIdx.x & 63;
    const int s = lane < d.E ? lane : d.E - 1;
#ifndef ZS_OBS_DIAG
#define ZS_OBS_DIAG 0
#endif
    const int ee = (ZS_OBS_DIAG & 4) ? 0 : e, ed = (ZS_OBS_DIAG & 2) ? 0 : e, eh = (ZS_OBS_DIAG & 1) ? 0 : e;
    f.pos = d.pos[EIX(d, s, ee)];
    f.life = d.life[EIX(d, s, ee)];
    f.wp = d.weapon[EIX(d, s, ee)];
    f.pr = d.present[EIX(d, s, ee)];
    const uint32_t* dr = d.dead + (size_t)ed * d.DW;
#pragma unroll
    for (int i = 0; i < OBS_PF_D; i++) {
        const int w = min(lane + 64 * i, d.DW - 1);
        f.dead[i] = (((dirty.y >> ((w * d.dead_chunk_m) >> 20)) & 1u) ? dr : d.dead_zero)[w];
    }
    // an obstacle is cleaned up only at life <= 0, so an env with no HP chunk dirty has every one
    f.opres = (dirty.x ? d.obst_present + (size_t)ed * d.OW : d.opres_full)[min(lane, max(d.OW - 1, 0))];
    const int32_t* hr = d.obst_hp + (size_t)eh * d.O;
#pragma unroll
    for (int i = 0; i < OBS_PF_H; i++) {
        const int o = min(lane + 64 * i, d.O - 1);
        f.hp[i] = (((dirty.x >> ((o * d.hp_chunk_m) >> 20)) & 1u) ? hr : d.hp_init)[o];
    }
}
__device__ __forceinline__ void obs_prefetch(const Dev& d, int e, int ahead, zs_v2u dirty, ObsPrefetch& f) {
    obs_prefetch_env(d, e, dirty, f);
    f.dirty_ahead = obs_dirty(d, ahead);
}

// The compact image (obs_cell_lds) of one env from its prefetched registers.  Lane l holds the HP of
// obstacles l, l + 64, ... and the present bits of obstacles 32l .. 32l + 31: obstacle o's bit comes
// from lane o >> 5 by a cross-lane read.
__device__ __forceinline__ void obs_build_compact(const Dev& d, const ObsLayout& L, lu8* img, const ObsPrefetch& f,
                                                  int code_s, int lane) {
    for (int w = lane; w < L.win / 4; w += 64) ((lu32*)img)[w] = 0u;
    if (lane < d.E) {
        ((li32*)(img + L.off_pos))[lane] = f.pos;
        ((lv2i*)(img + L.off_life))[lane] = zs_v2i{code_s | (f.wp << 8) | (f.pr << 16), f.life};
    }
    lu32* dead = (lu32*)(img + L.off_dead);
#pragma unroll
    for (int i = 0; i < OBS_PF_D; i++)
        if (lane + 64 * i < d.DW) dead[lane + 64 * i] = f.dead[i];
    li32* hpx = (li32*)(img + L.off_hp);
#pragma unroll
    for (int i = 0; i < OBS_PF_H; i++) {
        const uint32_t pw = (uint32_t)__shfl((int)f.opres, (lane >> 5) + 2 * i);
        if (lane + 64 * i < d.O) hpx[lane + 64 * i] = ((pw >> (lane & 31)) & 1u) ? f.hp[i] : ZS_HP_ABSENT;
    }
}

// window map of the compact image: every present entity's slot + 1 in each agent's window
template <int NOBS>
__device__ __forceinline__ void obs_window_compact(const Dev& d, const ObsLayout& L, lu8* img, int lane) {
    constexpr int WW = 21, PLANE = WW * WW;
    const li32* pos = (const li32*)(img + L.off_pos);
    const lv2i* ent = (const lv2i*)(img + L.off_life);
    if (lane < d.E && ((ent[lane].x >> 16) & 1)) {
        const int32_t p = pos[lane];
        const int x = unpack_x(p), y = unpack_y(p);
#pragma unroll
        for (int a = 0; a < NOBS; a++) {
            const int32_t ap = pos[a];
            const int dx = x - (unpack_x(ap) - WW / 2), dy = y - (unpack_y(ap) - WW / 2);
            if (dx >= 0 && dy >= 0 && dx < WW && dy < WW) img[a * PLANE + dy * WW + dx] = (uint8_t)(lane + 1);
        }
    }
}

template <typename T, int NOBS>
__global__ void __launch_bounds__(256, ZS_OBS_PIPE_WAVES) k_obs_pipe(Dev d, T* out, ObsLayout L, int env0, int env1) {
    if (blockIdx.x == 0 && threadIdx.x == 0) step_tail(d);  // a zs_step's tail (Dev::tail_*)
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr int WW = 21, PLANE = WW * WW, PER = (PLANE + 63) / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int stat_words = 4 * d.DW;
    lv4u* st4 = (lv4u*)smem;
    obs_stage_static4(d, st4, threadIdx.x, blockDim.x);
    __syncthreads();
    const int waves = gridDim.x * 4;
    int e = env0 + xcd_remap(blockIdx.x, gridDim.x) * 4 + wave;
    if (e >= env1) return;
    lu8* img = (lu8*)(smem + stat_words * 4 + wave * L.bytes);
    const li32* pos = (const li32*)(img + L.off_pos);
    const bool ch = d.obs_enc == ZS_ENC_CHANNELS;
    const int C = ch ? 3 : 1;
    const int code_s = lane < d.A ? (ch ? d.agent_codes[lane < d.A ? lane : 0] : ZS_THING_AGENT)
                                  : (lane < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
    ObsPrefetch f;
    obs_prefetch(d, e, min(e + waves, env1 - 1), OBS_OWN_ROWS, f);
    for (; e < env1; e += waves) {
        obs_build_compact(d, L, img, f, code_s, lane);  // the image of env e from the registers
        // the next env (the last wave re-reads its own), with the dirty masks its prefetch loaded
        const int en = min(e + waves, env1 - 1);
        obs_prefetch(d, en, min(en + waves, env1 - 1), f.dirty_ahead, f);
        wave_sync();
        obs_window_compact<NOBS>(d, L, img, lane);
        wave_sync();
        // the store stream
#pragma unroll 1
        for (int a = 0; a < NOBS; a++) {
            const int32_t ap = pos[a];
            const int ox = unpack_x(ap) - WW / 2, oy = unpack_y(ap) - WW / 2;
            const lu8* wm = img + a * PLANE;
            T* o = out + ((size_t)e * NOBS + a) * C * PLANE;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int cell = lane + 64 * i;
                const int cc = cell < PLANE ? cell : PLANE - 1;
                const int r = cc / WW, q = cc - r * WW;
                int code, lf, weapon;
                obs_cell_lds(d, L, st4, img, wm, cc, ox + q, oy + r, code, lf, weapon);
                if (cell < PLANE) obs_store(o, PLANE, cell, ch, code, lf, weapon);
            }
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// LDS-staged 16-B stores (k_obs_patch, k_obs_ring, k_obs_pbring): each observation block (3 x 441
// values, channels encoding) is first computed into an LDS slot, laid out at the destination's 16-B
// phase, and then streamed out as 16-B stores: every full 16-B chunk of the block is one aligned
// global_store_dwordx4 (half the store instructions of per-cell int64 stores, an eighth of int16 ones)
// and the stream carries no lookups between its stores; the partial chunks at the block's two ends are
// element stores.  tools/probe/storebw.hip: this store shape 6.0 TB/s.  The slot holds the values in the
// narrowest lossless type (obs_stage_t: int32 for int64 output — every channel value is an int32: codes,
// lives, weapon codes), widened by the flush, so an int64 block stages in 5.3 KB instead of 10.6 KB.
// (Round 6 removed k_obs_lds, k_obs_pipe's walk over this flush without writer waves: the ring and the
// padded-table kernel replaced it wherever it was the pick.)
// ---------------------------------------------------------------------------
template <typename T> struct obs_stage { typedef T type; };
template <> struct obs_stage<int64_t> { typedef int32_t type; };

// staging bytes: nblk consecutive channels blocks (one agent's, or every agent's of an env), shifted
// by the destination's 16-B phase in elements
__host__ __device__ constexpr int obs_stage_slot_bytes(int tsize, int nblk = 1) {
    return (((nblk * 3 * 441 + 16 / tsize) * (tsize == 8 ? 4 : tsize) + 15) / 16) * 16;
}

// Stream one staged block to o: slot element k + mis / sizeof(T) holds output element k, so the
// 16-B chunk q of the destination (counted from the 16-B boundary at or below o) reads the aligned
// slot elements [q * VPC, (q + 1) * VPC).
// Buffer-resource stores (raw buffer, gfx9 descriptor word 3): a lane whose offset is past the
// resource's range is dropped by the hardware, so a masked store needs no branch.  Every flush is then
// a fixed number of store instructions on every path, and the compiler's vmcnt waits for the next
// env's prefetch loads (issued before these stores, completing in order) count them exactly instead
// of assuming the shortest path and draining most of the stores still in flight.
#define ZS_OOB 0x80000000u

// base is wave-uniform at every caller (one block per wave); read through readfirstlane so the descriptor
// is built in SGPRs even where the compiler cannot prove that (k_obs_bring<int64, 4> wrapped each of its
// writers' buffer stores in a readfirstlane waterfall loop without it)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t zs_rsrc(void* base, uint32_t bytes) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0, (int)bytes, 0x00020000);
}
template <typename T>
__device__ __forceinline__ void zs_buf_store(__amdgpu_buffer_rsrc_t r, uint32_t off, T v) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t u = (uint64_t)v;
        __builtin_amdgcn_raw_buffer_store_b64(zs_v2u{(uint32_t)u, (uint32_t)(u >> 32)}, r, (int)off, 0, obs_aux<T>());
    } else if constexpr (sizeof(T) == 4) {
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, r, (int)off, 0, obs_aux<T>());
    } else {
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)v, r, (int)off, 0, obs_aux<T>());
    }
}

// Store throttle: at most ZS_OBS_THR of the wave's memory operations in flight after each 16-B store
// (-1: none).  HBM write bandwidth on this part falls when the whole chip keeps tens of thousands of
// 1-KB wave stores in flight (tools/probe/storeceil.hip: a flat 16-B store stream reaches 6.6-6.7
// TB/s with ~2-4 MB in flight chip-wide, 5.0-5.4 TB/s with 2048-4096 waves issuing unthrottled).
#ifndef ZS_OBS_THR
#define ZS_OBS_THR 2  // measured on one MI355X, C3 k_obs_lds 343 -> 315 us (4 runs each; vmcnt 1/3/4/6 no better)
#endif
#define ZS_STR2(x) #x
#define ZS_STR(x) ZS_STR2(x)
__device__ __forceinline__ void obs_store_throttle() {
#if ZS_OBS_THR >= 0
    asm volatile("s_waitcnt vmcnt(" ZS_STR(ZS_OBS_THR) ")" ::: "memory");
#endif
}

// Stream one staged block to o: slot element k + mis / sizeof(T) holds output element k, so the
// 16-B chunk q of the destination (counted from the 16-B boundary at or below o) reads the aligned
// slot elements [q * VPC, (q + 1) * VPC).  The partial chunks at the two ends are element stores.
// narrow (int16 / int32) blocks: C5's int16 stream moves a quarter of C3's bytes per cell and is not
// write-bound, so its flush need not hold stores back
#ifndef ZS_OBS_THR_NARROW
#define ZS_OBS_THR_NARROW ZS_OBS_THR
#endif
#ifndef ZS_FLUSH_GLOBAL
#define ZS_FLUSH_GLOBAL 1
#endif
template <typename T, int NBLK = 1, int THR = (sizeof(T) == 8 ? ZS_OBS_THR : ZS_OBS_THR_NARROW)>
__device__ __forceinline__ void obs_stage_flush(const lu8* slot, T* o, int lane) {
    typedef typename obs_stage<T>::type S;
    constexpr int TS = (int)sizeof(T), VPC = 16 / TS, NB = NBLK * 3 * 441 * TS;
    constexpr int NCH = (NB + 15 + 15) / 16;
    const int mis = (int)((uintptr_t)o & 15), shift = mis / TS;
    const ZS_LDS S* sv = (const ZS_LDS S*)slot;
    const __amdgpu_buffer_rsrc_t r = zs_rsrc(o, NB);
    const int nb = mis + NB, kend = nb >> 4, k0 = mis ? 1 : 0;
#pragma unroll
    for (int i = 0; i < (NCH + 63) / 64; i++) {
        const int k = lane + 64 * i;
        const int kr = k < kend ? k : kend - 1;
        zs_v4u v;
        if constexpr (TS == 8) {  // two int32 -> two int64
            const zs_v2u w = *(const ZS_LDS zs_v2u*)(sv + kr * VPC);
            v = zs_v4u{w.x, (uint32_t)((int32_t)w.x >> 31), w.y, (uint32_t)((int32_t)w.y >> 31)};
        } else {
            v = *(const ZS_LDS zs_v4u*)(sv + kr * VPC);
        }
        if (ZS_FLUSH_GLOBAL) {
            // plain global stores of the whole 16-B chunks: on this part a stream of them runs 6 % faster than the
            // same stream of raw buffer stores (tools/probe/storepat2.hip, profiles/r05k_storepat2.log)
            if (k >= k0 && k < kend) {
                zs_v4u* dst = (zs_v4u*)((uint8_t*)o - mis) + k;
                if constexpr (obs_aux<T>() != 0) __builtin_nontemporal_store(v, dst);
                else *dst = v;
            }
        } else {
            __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)((k >= k0 && k < kend) ? (uint32_t)(16 * k - mis) : ZS_OOB), 0,
                                                   obs_aux<T>());
        }
        if (THR >= 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(THR < 0 ? 0 : THR) : "memory");
    }
    const int nhead = mis ? (16 - mis) / TS : 0, tail0 = (16 * kend - mis) / TS, ntail = (nb - 16 * kend) / TS;
    const int idx = lane < nhead ? lane : (lane >= 32 && lane - 32 < ntail) ? tail0 + lane - 32 : -1;
    zs_buf_store<T>(r, idx >= 0 ? (uint32_t)(idx * TS) : ZS_OOB, (T)sv[(idx >= 0 ? idx : 0) + shift]);
}

// ---------------------------------------------------------------------------
// k_obs_gather: the registered shape (surroundings, width 21, NOBS observations per env) on maps
// whose obstacle HP row is too large to stage per env (city128: 3689 obstacles, 14.7 KB, which
// left k_obs one wave per CU slot).  Only the observed cells' data is fetched: per lane, the
// static per-cell words of its NOBS x 7 window cells, then the HP of those cells' obstacles, each
// batch issued as one group of loads before any store (one wait per batch, no global load inside
// the store loop).  The wave image holds the window maps, entities, dead-body and obstacle-present
// bits only (~5 KB at city128), so four waves per workgroup and many workgroups per CU hide the two
// load round trips.
// ---------------------------------------------------------------------------
// stat (uniform): the map's static tables (obs_stage_static4, 16 * DW bytes at the start of the
// workgroup's LDS) give each window cell's static word (obstacle rank, kind, objective bit) by LDS
// reads, so the HP loads follow the env's first load round directly (two dependent load rounds
// instead of three).
template <typename T, int NOBS>
__global__ void __launch_bounds__(256) k_obs_gather(Dev d, T* out, const uint8_t* mask, ObsLayout L, int stat) {
    if (blockIdx.x == 0 && threadIdx.x == 0) step_tail(d);  // a zs_step's tail (Dev::tail_*)
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr int WW = 21, PLANE = WW * WW, PER = (PLANE + 63) / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int e = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave;
    const bool act = e < d.N && !(mask && !mask[e]);
    if (!stat && !act) return;
    const lv4u* st4 = (const lv4u*)smem;
    lu8* img = (lu8*)(smem + (stat ? 16 * d.DW : 0) + wave * L.bytes);
    const int W = d.W, H = d.H;
    if (stat) obs_stage_static4(d, (lv4u*)smem, threadIdx.x, blockDim.x);
    uint32_t hpd = 0;  // arrives with obs_build's loads, used one load round later
    if (act) {
        hpd = d.hp_dirty[e];
        obs_build(d, L, img, e, [&](int s, int& p, int& lf, int& wp, int& pr) {
            p = d.pos[EIX(d, s, e)];
            lf = d.life[EIX(d, s, e)];
            wp = d.weapon[EIX(d, s, e)];
            pr = d.present[EIX(d, s, e)];
        });
    }
    if (stat) __syncthreads();
    if (!act) return;
    const li32* pos = (const li32*)(img + L.off_pos);
    const li32* life = (const li32*)(img + L.off_life);
    const li32* cw = (const li32*)(img + L.off_cw);
    const lu32* dead = (const lu32*)(img + L.off_dead);
    const lu32* opres = (const lu32*)(img + L.off_opres);
    const bool ch = d.obs_enc == ZS_ENC_CHANNELS;
    const int C = ch ? 3 : 1;
    const int32_t* hrow = d.obst_hp + (size_t)e * d.O;
    uint32_t sc[NOBS][PER];
    int32_t hv[NOBS][PER];
    // static words of the window cells (out-of-bounds cells read cell 0, discarded below)
#pragma unroll
    for (int a = 0; a < NOBS; a++) {
        const int32_t ap = pos[a];
        const int ox = unpack_x(ap) - WW / 2, oy = unpack_y(ap) - WW / 2;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int cc = min(lane + 64 * i, PLANE - 1), r = cc / WW, q = cc - r * WW;
            const int x = ox + q, y = oy + r;
            const bool inb = (unsigned)x < (unsigned)W && (unsigned)y < (unsigned)H;
            const int c = inb ? y * W + x : 0;
            if (stat) {  // the scell word (engine.hip) from the static tables
                const uint32_t bit = 1u << (c & 31);
                const zs_v4u sw = st4[c >> 5];
                const uint32_t ob = (sw.x & bit) ? (sw.w + __popc(sw.x & (bit - 1u)) + 1u) |
                                                       ((uint32_t)((sw.y & bit) ? ZS_THING_BOX : ZS_THING_WALL) << SC_KIND_SHIFT)
                                                 : 0u;
                sc[a][i] = ob | ((sw.z & bit) ? SC_OBJ_BIT : 0u);
            } else {
                sc[a][i] = (uint32_t)d.scell[c];
            }
        }
    }
    // HP of the window cells' obstacles (cells without one read obstacle 0, discarded below); a clean
    // chunk's HP from the shared hp_init row
    const uint32_t dirty = hpd;
#pragma unroll
    for (int a = 0; a < NOBS; a++)
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int oi = (int)(sc[a][i] & SC_OBST_MASK) - 1;
            const int o = oi > 0 ? oi : 0;
            hv[a][i] = (((dirty >> (o / d.hp_chunk)) & 1u) ? hrow : d.hp_init)[o];
        }
    // the store stream: LDS and registers only
#pragma unroll 1
    for (int a = 0; a < NOBS; a++) {
        const int32_t ap = pos[a];
        const int ox = unpack_x(ap) - WW / 2, oy = unpack_y(ap) - WW / 2;
        const lu8* wm = img + a * PLANE;
        T* o = out + ((size_t)e * NOBS + a) * C * PLANE;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int cell = lane + 64 * i;
            const int cc = cell < PLANE ? cell : PLANE - 1, r = cc / WW, q = cc - r * WW;
            const int x = ox + q, y = oy + r;
            const bool inb = (unsigned)x < (unsigned)W && (unsigned)y < (unsigned)H;
            const int c = inb ? y * W + x : 0;
            const uint32_t bit = 1u << (c & 31);
            const int sb = wm[cc];
            const int v = cw[sb ? sb - 1 : 0], elife = life[sb ? sb - 1 : 0];
            const uint32_t s = sc[a][i];
            const int oi = (int)(s & SC_OBST_MASK) - 1;
            const bool obp = oi >= 0 && ((opres[(oi > 0 ? oi : 0) >> 5] >> (oi & 31)) & 1u);
            int code = (dead[c >> 5] & bit) ? ZS_THING_DEADBODY : (s & SC_OBJ_BIT) ? ZS_THING_OBJECTIVE : ZS_THING_NONE;
            code = obp ? (int)((s >> SC_KIND_SHIFT) & 7u) : code;
            code = sb ? (v & 255) : code;
            code = inb ? code : ZS_THING_WALL;
            int lf = sb ? elife : (obp ? hv[a][i] : 0);
            lf = inb ? lf : 200;
            const int weapon = (inb && sb) ? ((v >> 8) & 255) : 0;
            if (cell < PLANE) obs_store(o, PLANE, cell, ch, code, lf, weapon);
        }
    }
}

// ---------------------------------------------------------------------------
// k_obs_patch: k_obs_pipe's walk and two-env prefetch with the LDS-staged 16-B flush and a cheaper encoder.  A window cell's
// value is first taken from a padded static table of the map (one LDS read: the code and life the
// cell shows when no thing stands on it, every obstacle is present at its MAX_LIFE and no body lies
// there; out-of-bounds cells are Wall(200) entries of the padding), then the few cells whose value
// differs are patched in place, in rising precedence (gym/observation.py:57-90: thing > present
// obstacle > dead body > objective > empty):
//   * obstacles whose life left MAX_LIFE or that were cleaned up (core.py:121-138): a per-env list in
//     LDS, compacted once per env, each entry the cell and the value it shows;
//   * dead bodies on cells without a map obstacle, from the env's dead-body words in registers;
//   * the present things, one per lane (slot s on lane s).
// Per cell that is one LDS read and three slot writes instead of k_obs_lds's five dependent lookups and
// select chain (C5: ~51 VALU instructions per cell, the kernel VALU-issue-bound at 63 % busy).
// ---------------------------------------------------------------------------
// padded table entry (engine.hip: opad): bits 0..2 the code, bit 3 objective under a map obstacle,
// bits 8..15 the life; opk (per obstacle): x | y << 12 | box << 24 | objective-under << 25
#define OPAD_OBJ 8u
__host__ __device__ constexpr int patch_list_bytes(int O) { return ((O * 8 + 15) / 16) * 16; }
// static LDS of a workgroup: the padded table and the obstacles' packed cells
__host__ __device__ constexpr int patch_static_bytes(int opad_n, int O) {
    return ((opad_n * 2 + 15) / 16) * 16 + ((O * 4 + 15) / 16) * 16 + 256;
}

// per-env list of dead-body cells (without a map obstacle) the encoder patches; an env with more takes
// the per-word scan
#define PATCH_DEAD_CAP 256
__host__ __device__ constexpr int patch_enc_bytes(int DW, int O) {  // dead words, present words, dead list, list
    return ((DW * 4 + 15) / 16) * 16 + 256 + 4 * PATCH_DEAD_CAP + 16 + patch_list_bytes(O);
}
__host__ __device__ constexpr int patch_wave_bytes(int DW, int O, int slot) { return patch_enc_bytes(DW, O) + slot; }

// Stage the static tables into the workgroup's LDS (all threads, then a barrier): the padded table,
// the obstacles' packed cells, and per lane the Box bits of its obstacles lane + 64 i.
__device__ __forceinline__ void patch_stage_static(const Dev& d, uint8_t* smem) {
    const int padb = ((d.opad_n * 2 + 15) / 16) * 16, okb = ((d.O * 4 + 15) / 16) * 16;
    const zs_v4u* src = (const zs_v4u*)d.opad;
    lv4u* dst = (lv4u*)smem;
    for (int k = threadIdx.x; k < padb / 16; k += blockDim.x) dst[k] = src[k];
    lu32* ok = (lu32*)(smem + padb);
    for (int k = threadIdx.x; k < d.O; k += blockDim.x) ok[k] = d.opk[k];
    __syncthreads();
    if (threadIdx.x < 64) {
        uint32_t m = 0u;
        for (int i = 0; i < OBS_PF_H; i++) m |= ((d.opk[min((int)threadIdx.x + 64 * i, d.O - 1)] >> 24) & 1u) << i;
        ((lu32*)(smem + padb + okb))[threadIdx.x] = m;
    }
    __syncthreads();
}

// One wave's encoder: the env it encodes held in registers (lane s: entity slot s), its dead-body
// words, obstacle-present words and obstacle list in the wave's LDS region `wb` (patch_enc_bytes).
template <typename S>
struct PatchEnc {
    static constexpr int WW = 21, HALF = WW / 2, PLANE = WW * WW, PER = (PLANE + 63) / 64;
    const lu16* pad;
    const lu32* okl;
    const lu32* boxl;
    lu32* deadl;
    lu32* presl;
    lu32* dlist;  // dead-body cells x | y << 16
    lu32* dcnt;
    ZS_LDS zs_v2i* lst;
    int lane, PW, W, code_s;
    // per lane, for the whole walk: its window cells' offsets in the padded table from a window's
    // corner, two 16-bit offsets per register (engine.hip admits the kernel when 21 rows < 65536)
    uint32_t offp[(PER + 1) / 2];
    int32_t pos, life;
    int wp, pr;
    int nchg;       // entries of the obstacle list (wave-uniform)
    int ndead;      // entries of the dead-body list, -1: more than PATCH_DEAD_CAP (wave-uniform)
    bool any_dead;  // some dead-body word is non-zero (wave-uniform)

    __device__ __forceinline__ PatchEnc(const Dev& d, uint8_t* smem, lu8* wb, int lane_) : lane(lane_) {
        const int padb = ((d.opad_n * 2 + 15) / 16) * 16, okb = ((d.O * 4 + 15) / 16) * 16;
        pad = (const lu16*)smem;
        okl = (const lu32*)(smem + padb);
        boxl = (const lu32*)(smem + padb + okb);
        deadl = (lu32*)wb;
        presl = (lu32*)(wb + ((d.DW * 4 + 15) / 16) * 16);  // OW <= 64
        dlist = (lu32*)(wb + ((d.DW * 4 + 15) / 16) * 16 + 256);
        dcnt = dlist + PATCH_DEAD_CAP;
        lst = (ZS_LDS zs_v2i*)(wb + ((d.DW * 4 + 15) / 16) * 16 + 256 + 4 * PATCH_DEAD_CAP + 16);
        PW = d.opad_w;
        W = d.W;
        code_s = lane < d.A ? d.agent_codes[lane < d.A ? lane : 0] : (lane < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int cc = min(lane + 64 * i, PLANE - 1), r = cc / WW;
            const uint32_t v = (uint32_t)(r * PW + (cc - r * WW));
            if (i % 2 == 0) offp[i / 2] = v;
            else offp[i / 2] |= v << 16;
        }
    }

    // a prefetched env's registers -> this encoder; its dead-body words and obstacle list -> LDS
    __device__ __forceinline__ void build(const Dev& d, const ObsPrefetch& f) {
        pos = f.pos;
        life = f.life;
        wp = f.wp;
        pr = f.pr;
        bool nz = false;
#pragma unroll
        for (int i = 0; i < OBS_PF_D; i++)
            if (lane + 64 * i < d.DW) {
                deadl[lane + 64 * i] = f.dead[i];
                nz |= f.dead[i] != 0u;
            }
        any_dead = __ballot(nz) != 0ull;
        ndead = 0;
        if (any_dead) {
            // the env's dead-body cells that no map obstacle covers (a map obstacle's cell is the obstacle
            // list's business), compacted once for every agent's window
            if (lane == 0) *dcnt = 0u;
            wave_sync();
#pragma unroll
            for (int i = 0; i < OBS_PF_D; i++) {
                const int w = lane + 64 * i;
                uint32_t bits = w < d.DW ? f.dead[i] : 0u;
                if (bits) {
                    uint32_t k = __hip_atomic_fetch_add(dcnt, (uint32_t)__popc(bits), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    while (bits) {
                        const int c = 32 * w + __ffs(bits) - 1;
                        bits &= bits - 1u;
                        const int y = d.w_m ? (int)(((uint32_t)c * d.w_m) >> 20) : c / W, x = c - y * W;
                        const uint32_t sc = pad[(y + HALF) * PW + x + HALF] & 7u;
                        if (sc != ZS_THING_BOX && sc != ZS_THING_WALL) {
                            if (k < PATCH_DEAD_CAP) dlist[k] = (uint32_t)x | ((uint32_t)y << 16);
                            k++;
                        } else {
                            dlist[k < PATCH_DEAD_CAP ? k : 0] = 0xffffffffu;  // a hole: matches no window
                            k++;
                        }
                    }
                }
            }
            wave_sync();
            const int n = (int)__builtin_amdgcn_readfirstlane(*dcnt);
            ndead = n <= PATCH_DEAD_CAP ? n : -1;
        }
        // obstacles away from the table's value: life off MAX_LIFE, or cleaned up.  The Box bits are read
        // back per env rather than held (a loop-invariant register set the compiler would spill).
        const int ow = min(lane, max(d.OW - 1, 0)), nb = min(32, d.O - 32 * ow);
        const uint32_t full = nb == 32 ? 0xffffffffu : ((1u << nb) - 1u);
        bool odd = lane < d.OW && f.opres != full;
        const uint32_t boxm = boxl[lane];
#pragma unroll
        for (int i = 0; i < OBS_PF_H; i++) odd |= lane + 64 * i < d.O && f.hp[i] != (((boxm >> i) & 1u) ? 10 : 200);
        nchg = 0;
        if (__ballot(odd) == 0ull) return;
        if (lane < d.OW) presl[lane] = f.opres;
        wave_sync();  // the dead-body and present words before the lookups below
        int n = 0;
#pragma unroll
        for (int i = 0; i < OBS_PF_H; i++) {
            const uint32_t pw = presl[(lane >> 5) + 2 * i];  // past OW: unused (chg needs o < O)
            const bool pres = (pw >> (lane & 31)) & 1u;
            const uint32_t k = okl[lane + 64 * i];  // past O: another region's word, unused
            const bool box = (k >> 24) & 1u;
            const bool chg = lane + 64 * i < d.O && (!pres || f.hp[i] != (box ? 10 : 200));
            const unsigned long long m = __ballot(chg);
            if (chg) {
                const int x = (int)(k & 0xfffu), y = (int)((k >> 12) & 0xfffu), c = y * W + x;
                int code = ((k >> 25) & 1u) ? ZS_THING_OBJECTIVE : ZS_THING_NONE;
                code = ((deadl[c >> 5] >> (c & 31)) & 1u) ? ZS_THING_DEADBODY : code;
                code = pres ? (box ? ZS_THING_BOX : ZS_THING_WALL) : code;
                lst[n + __popcll(m & ((1ull << lane) - 1ull))] = zs_v2i{(int)(k & 0xffffffu) | (code << 24), pres ? f.hp[i] : 0};
            }
            n += __popcll(m);
        }
        nchg = n;
    }

    // agent a's 3 x 21 x 21 block into ot (elements of S)
    __device__ __forceinline__ void block(const Dev& d, ZS_LDS S* ot, int a) const {
        const int32_t ap = __builtin_amdgcn_readlane(pos, a);
        const int ax = unpack_x(ap), ay = unpack_y(ap);
        const int pbase = ay * PW + ax;  // padded cell of the window's corner (ax - HALF, ay - HALF)
#pragma unroll
        for (int i = 0; i < ((ZS_OBS_DIAG & 16) ? 0 : PER); i++) {  // diagnostic builds: 16 skips the encoding
            const int cell = lane + 64 * i;
            if (i + 1 < PER || cell < PLANE) {
                const uint32_t v = pad[pbase + (int)((offp[i / 2] >> (16 * (i % 2))) & 0xffffu)];
                ot[cell] = (S)(v & 7u);
                ot[PLANE + cell] = (S)(v >> 8);
                ot[2 * PLANE + cell] = (S)0;
            }
        }
        // obstacles off the table's value
        for (int k = lane; k < nchg; k += 64) {
            const zs_v2i en = lst[k];
            const int dx = (en.x & 0xfff) - ax + HALF, dy = ((en.x >> 12) & 0xfff) - ay + HALF;
            if ((unsigned)dx < (unsigned)WW && (unsigned)dy < (unsigned)WW) {
                const int cc = dy * WW + dx;
                ot[cc] = (S)((en.x >> 24) & 7);
                ot[PLANE + cc] = obs_val<S>(en.y);
            }
        }
        // dead bodies on cells without a map obstacle (a map obstacle's cell is the list's business)
        for (int k = lane; k < ((ZS_OBS_DIAG & 32) ? 0 : ndead); k += 64) {  // diagnostic builds: 32 skips them
            const uint32_t en = dlist[k];
            const int dx = (int)(en & 0xffffu) - ax + HALF, dy = (int)(en >> 16) - ay + HALF;
            if ((unsigned)dx < (unsigned)WW && (unsigned)dy < (unsigned)WW) {
                const int cc = dy * WW + dx;
                ot[cc] = (S)ZS_THING_DEADBODY;
                ot[PLANE + cc] = (S)0;
            }
        }
        if (ndead < 0 && !(ZS_OBS_DIAG & 32)) {  // more bodies than the list holds: the per-word scan
            const int c_lo = (ay - HALF) * W, c_hi = (ay + HALF + 1) * W;  // the window's rows
            // maps whose rows are whole words: the window's columns as a mask of each word's bits
            const int x0 = ax - HALF, wpr = W >> 5;
            const bool rowwords = (W & 31) == 0;
#pragma unroll
            for (int i = 0; i < OBS_PF_D; i++) {
                const int w = lane + 64 * i;
                uint32_t bits = w < d.DW ? deadl[w] : 0u;
                if (32 * w + 31 < c_lo || 32 * w >= c_hi) bits = 0u;
                if (rowwords) {  // columns [x0 - base, x0 - base + 21) of this word's 32
                    const int lo = x0 - 32 * (w - (w / wpr) * wpr);
                    const uint32_t m_hi = lo + WW >= 32 ? 0xffffffffu : (lo + WW <= 0 ? 0u : ((1u << (lo + WW)) - 1u));
                    const uint32_t m_lo = lo <= 0 ? 0xffffffffu : (lo >= 32 ? 0u : ~((1u << lo) - 1u));
                    bits &= m_hi & m_lo;
                }
                while (bits) {
                    const int c = 32 * w + __ffs(bits) - 1;
                    bits &= bits - 1u;
                    const int y = d.w_m ? (int)(((uint32_t)c * d.w_m) >> 20) : c / W, x = c - y * W;
                    const int dx = x - ax + HALF, dy = y - ay + HALF;
                    if ((unsigned)dx < (unsigned)WW && (unsigned)dy < (unsigned)WW) {
                        const uint32_t sc = pad[(y + HALF) * PW + x + HALF] & 7u;
                        if (sc != ZS_THING_BOX && sc != ZS_THING_WALL) {
                            const int cc = dy * WW + dx;
                            ot[cc] = (S)ZS_THING_DEADBODY;
                            ot[PLANE + cc] = (S)0;
                        }
                    }
                }
            }
        }
        // the present things
        if (lane < d.E && pr) {
            const int dx = unpack_x(pos) - ax + HALF, dy = unpack_y(pos) - ay + HALF;
            if ((unsigned)dx < (unsigned)WW && (unsigned)dy < (unsigned)WW) {
                const int cc = dy * WW + dx;
                ot[cc] = (S)code_s;
                ot[PLANE + cc] = obs_val<S>(life);
                ot[2 * PLANE + cc] = (S)wp;
            }
        }
    }
};

// waves per workgroup: eight share one copy of the static tables (16 KB at bridge64), two workgroups
// per CU
#define PATCH_WPG 8
template <typename T, int NOBS>
__global__ void __launch_bounds__(64 * PATCH_WPG, ZS_OBS_PIPE_WAVES) k_obs_patch(Dev d, T* out, int env0, int env1) {
    if (blockIdx.x == 0 && threadIdx.x == 0) step_tail(d);  // a zs_step's tail (Dev::tail_*)
    extern __shared__ __align__(16) uint8_t smem[];
    typedef typename obs_stage<T>::type S;
    constexpr int PLANE = 441, TS = (int)sizeof(T), SLOT = obs_stage_slot_bytes(TS);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    patch_stage_static(d, smem);
    const int waves = gridDim.x * PATCH_WPG;
    int e = env0 + xcd_remap(blockIdx.x, gridDim.x) * PATCH_WPG + wave;
    if (e >= env1) return;
    lu8* wb = (lu8*)(smem + patch_static_bytes(d.opad_n, d.O) + wave * patch_wave_bytes(d.DW, d.O, SLOT));
    lu8* slot = wb + patch_enc_bytes(d.DW, d.O);  // 16-B aligned
    PatchEnc<S> pe(d, smem, wb, lane);
    auto process = [&](int e) __attribute__((always_inline)) {
#pragma unroll
        for (int a = 0; a < NOBS; a++) {
            T* o = out + ((size_t)e * NOBS + a) * 3 * PLANE;
            pe.block(d, (ZS_LDS S*)slot + (int)((uintptr_t)o & 15) / TS, a);
            wave_sync();
            if (!(ZS_OBS_DIAG & 8)) obs_stage_flush(slot, o, lane);
            wave_sync();
        }
    };
    // two envs of register prefetch in flight, as k_obs_lds
    ObsPrefetch fa, fb;
    {
        const int e1 = min(e + waves, env1 - 1);
        obs_prefetch(d, e, min(e + 2 * waves, env1 - 1), OBS_OWN_ROWS, fa);
        obs_prefetch(d, e1, min(e1 + 2 * waves, env1 - 1), obs_dirty(d, e1), fb);
    }
    pe.build(d, fa);
    for (;;) {
        {
            const int en = min(e + 2 * waves, env1 - 1);
            obs_prefetch(d, en, min(en + 2 * waves, env1 - 1), fa.dirty_ahead, fa);
        }
        process(e);
        e += waves;
        if (e >= env1) break;
        pe.build(d, fb);
        {
            const int en = min(e + 2 * waves, env1 - 1);
            obs_prefetch(d, en, min(en + 2 * waves, env1 - 1), fb.dirty_ahead, fb);
        }
        process(e);
        e += waves;
        if (e >= env1) break;
        pe.build(d, fa);
    }
}

// ---------------------------------------------------------------------------
// k_obs_ring: the LDS-staged flush with the encoding and the store stream on different waves.  A workgroup of
// RING_ENC encoder waves and RING_WRT writer waves walks envs b, b + G, ... (b = its XCD-contiguous
// index, G = the grid); encoder waves build an env's image from prefetched registers and encode every
// agent's block side by side into a ring slot of LDS (at the env's 16-B phase), writer waves stream
// whole envs from the ring as 16-B stores.  Only RING_WRT waves per CU store, so the chip keeps fewer
// streams in flight (tools/probe/storeceil.hip: one contiguous block per wave reaches 5.3 TB/s at 2048
// storing waves, 5.7 at 1024), and the encoders never wait on their own stores.
// The ring's unit is one env, or two adjacent envs when that makes the unit's output 16-B aligned
// (ring_pair); a unit's envs are encoded by different encoder waves into one slot and streamed out
// by one writer as one contiguous block.
// Slot protocol (LDS, this workgroup only): per slot q and env h of the unit, state = 2u + 1 once env
// h of unit u (q = u % slots) is encoded, 2u + 2 once the unit is streamed out; the encoder of unit
// u first waits for 2(u - slots) + 2.  Both sides walk upwards, so the smallest unencoded env always
// has its slot drained eventually: no wait cycle.  Every wave leaves after its last env.
// ---------------------------------------------------------------------------
#ifndef RING_ENC
#define RING_ENC 12
#endif
#ifndef RING_WRT
#define RING_WRT 3  // measured on one MI355X at C3 (2 runs each): 3 writers 267.7 / 269.0 us, 4: 273.4 / 274.4, 2: 282.8 / 283.6
#endif
#ifndef RING_SLOTS
#define RING_SLOTS 8
#endif
#ifndef RING_THR
#define RING_THR 16
#endif
#ifndef ZS_RING_PF
#define ZS_RING_PF 2  // encoder prefetch depth (items)
#endif
// Envs per ring unit: two when one env's block ends off a 16-B boundary and two end on one (C5's
// int16 10 584-B envs): a unit is then one aligned, contiguous stream, with no partial 16-B chunk
// shared by two writers.
__host__ __device__ constexpr int ring_pair(int tsize, int nobs) {
    return (nobs * 3 * 441 * tsize) % 16 != 0 && (2 * nobs * 3 * 441 * tsize) % 16 == 0 ? 2 : 1;
}
__host__ __device__ constexpr int ring_lds_bytes(int stat_bytes, int img_bytes, int tsize, int nobs) {
    return stat_bytes + RING_ENC * img_bytes +
           (RING_SLOTS / ring_pair(tsize, nobs)) * obs_stage_slot_bytes(tsize, nobs * ring_pair(tsize, nobs)) +
           16 * RING_SLOTS;
}

// The hand-off is LDS-only: a wave's LDS operations complete in order, so waiting for its own LDS
// traffic (lgkmcnt(0)) before the state store orders the slot's data before the state, and a reader's
// LDS reads after it sees the state see the data.  No memory fence: a workgroup release would also wait
// for the writer's global stores still in flight (vmcnt), which is the stream this kernel keeps going.
__device__ __forceinline__ int ring_state_load(const ZS_LDS int* p) { return *(const volatile ZS_LDS int*)p; }
__device__ __forceinline__ void ring_state_store(ZS_LDS int* p, int v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    *(volatile ZS_LDS int*)p = v;
}
__device__ __forceinline__ void ring_wait(const ZS_LDS int* p, int v) {
    while (ring_state_load(p) != v) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// PATCHED: the encoders are k_obs_patch's (PatchEnc), static tables patch_static_bytes, encoder regions
// patch_enc_bytes (ring_patch_lds_bytes)
__host__ __device__ constexpr int ring_patch_lds_bytes(int static_bytes, int enc_bytes, int tsize, int nobs) {
    return ring_lds_bytes(static_bytes, enc_bytes, tsize, nobs);
}
#ifndef ZS_RING_LAUNDER
#define ZS_RING_LAUNDER 1
#endif
// Dev is the first argument (zs_launder_dev's contract: the encoders reload it from kernarg offset 0)
template <typename T, int NOBS, bool PATCHED = false>
__global__ void __launch_bounds__(64 * (RING_ENC + RING_WRT), 1) k_obs_ring(Dev d, T* out, ObsLayout L, int env0, int env1) {
    const Dev& d0 = d;
    if (blockIdx.x == 0 && threadIdx.x == 0) step_tail(d);  // a zs_step's tail (Dev::tail_*)
    extern __shared__ __align__(16) uint8_t smem[];
    typedef typename obs_stage<T>::type S;
    constexpr int WW = 21, PLANE = WW * WW, TS = (int)sizeof(T);
    constexpr int PAIR = ring_pair(TS, NOBS), US = RING_SLOTS / PAIR;  // envs per unit, unit slots
    constexpr int SLOT = obs_stage_slot_bytes(TS, NOBS * PAIR), BLK = NOBS * 3 * PLANE;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int stat_bytes = PATCHED ? patch_static_bytes(d.opad_n, d.O) : 16 * d.DW;
    const int enc_bytes = PATCHED ? patch_enc_bytes(d.DW, d.O) : L.bytes;
    lv4u* st4 = (lv4u*)smem;
    lu8* slots = (lu8*)(smem + stat_bytes + RING_ENC * enc_bytes);
    // state[PAIR * slot + h]: the protocol word of the unit's env h
    ZS_LDS int* state = (ZS_LDS int*)(slots + US * SLOT);
    if (threadIdx.x < RING_SLOTS) state[threadIdx.x] = 0;
    if (PATCHED) {
        patch_stage_static(d, smem);
    } else {
        obs_stage_static4(d, st4, threadIdx.x, blockDim.x);
        __syncthreads();
    }
    // unit g covers envs env0 + PAIR * g + h (h < PAIR, below env1); this workgroup's units are
    // g_first, g_first + G, ...; its items (envs) t = PAIR * u + h, the last one possibly absent
    const int G = gridDim.x, n_units = (env1 - env0 + PAIR - 1) / PAIR;
#if ZS_RING_DEAL
    const XcdDeal deal(blockIdx.x, G, n_units, RING_WRT);
    const int ucount = deal.ucount;
    auto unit_of = [&](int u) { return deal.unit(u); };
#else
    const int g_first = xcd_remap(blockIdx.x, G);
    const int ucount = g_first < n_units ? (n_units - g_first + G - 1) / G : 0;
    auto unit_of = [&](int u) { return g_first + u * G; };
#endif
    // items in the last unit: PAIR, or fewer for the run's last unit
    const int count = ucount ? PAIR * (ucount - 1) + min(PAIR, env1 - env0 - PAIR * unit_of(ucount - 1)) : 0;
    auto unit_env = [&](int u) { return env0 + PAIR * unit_of(u); };
    if (wave >= RING_ENC) {  // writer
        for (int u = wave - RING_ENC; u < ucount; u += RING_WRT) {
            const int q = u % US, e = unit_env(u);
            const bool whole = PAIR * u + PAIR <= count;
            for (int h = 0; h < PAIR; h++)
                if (PAIR * u + h < count) ring_wait(&state[PAIR * q + h], 2 * u + 1);
            if (!(ZS_OBS_DIAG & 8)) {
                if (whole) obs_stage_flush<T, NOBS * PAIR, RING_THR>(slots + q * SLOT, out + (size_t)e * BLK, lane);
                else obs_stage_flush<T, NOBS, RING_THR>(slots + q * SLOT, out + (size_t)e * BLK, lane);
            }
            for (int h = 0; h < PAIR; h++) ring_state_store(&state[PAIR * q + h], 2 * u + 2);
        }
        return;
    }
    // encoder
    lu8* img = (lu8*)(smem + stat_bytes + wave * enc_bytes);
    PatchEnc<S> pe(d, smem, img, lane);
    const li32* pos = (const li32*)(img + L.off_pos);
    const int code_s = lane < d.A ? d.agent_codes[lane < d.A ? lane : 0] : (lane < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
    auto item_env = [&](int t) { return unit_env(t / PAIR) + t % PAIR; };
    int t = wave;
    if (t >= count) return;
    // encode item t: its image from f, then (before any LDS work) the loads of the item `ahead`
    // iterations later into f, with that item's dirty masks dq (loaded two iterations earlier), and
    // dq reloaded for the item two iterations after that
    auto encode = [&](int t, ObsPrefetch& f, zs_v2u& dq, int ahead) {
        // the Dev fields reloaded per item (ZS_RING_LAUNDER), not held in SGPRs across the wave's items
        const Dev& d = ZS_RING_LAUNDER ? *zs_launder_dev(d0) : d0;
        const int u = t / PAIR, h = t % PAIR, e = item_env(t);
        if (PATCHED) pe.build(d, f);
        else obs_build_compact(d, L, img, f, code_s, lane);
        // this item's prefetch set next serves item t + ahead * RING_ENC, whose loads need the dirty masks of
        // the item after that (t + 2 * ahead * RING_ENC)
        const int tn = t + ahead * RING_ENC, tq = t + 2 * ahead * RING_ENC;
        if (ahead == 1) {
            if (tn < count) obs_prefetch(d, item_env(tn), tn + RING_ENC < count ? item_env(tn + RING_ENC) : item_env(tn), f.dirty_ahead, f);
        } else {
            // every load unconditional (an item past the wave's last reads the wave's first env again),
            // so the waits for the older prefetch count the younger one's loads exactly
            obs_prefetch_env(d, item_env(tn < count ? tn : wave), dq, f);
            dq = obs_dirty(d, item_env(tq < count ? tq : wave));
        }
        wave_sync();
        if (!PATCHED) obs_window_compact<NOBS>(d, L, img, lane);
        const int q = u % US;
        if (u >= US) ring_wait(&state[PAIR * q + h], 2 * (u - US) + 2);
        wave_sync();
        ZS_LDS S* ot0 = (ZS_LDS S*)(slots + q * SLOT) + (int)((uintptr_t)(out + (size_t)(e - h) * BLK) & 15) / TS + h * BLK;
#pragma unroll
        for (int a = 0; a < ((ZS_OBS_DIAG & 16) ? 0 : NOBS); a++) {
            if (PATCHED) {
                pe.block(d, ot0 + a * 3 * PLANE, a);
            } else {
                const int32_t ap = pos[a];
                const int ox = unpack_x(ap) - WW / 2, oy = unpack_y(ap) - WW / 2;
                const lu8* wm = img + a * PLANE;
                obs_encode_block<S>(d, L, st4, img, wm, ox, oy, ot0 + a * 3 * PLANE, lane);
            }
        }
        ring_state_store(&state[PAIR * q + h], 2 * u + 1);
    };
    auto envc = [&](int tt) { return item_env(tt < count ? tt : wave); };
#if ZS_RING_PF == 2
    // two items of register prefetch: a load round trip under the saturated store stream outlasts the
    // encoding of one env
    ObsPrefetch fa, fb;
    zs_v2u qa, qb;
    obs_prefetch_env(d, envc(t), OBS_OWN_ROWS, fa);
    obs_prefetch_env(d, envc(t + RING_ENC), obs_dirty(d, envc(t + RING_ENC)), fb);
    qa = obs_dirty(d, envc(t + 2 * RING_ENC));
    qb = obs_dirty(d, envc(t + 3 * RING_ENC));
    for (; t < count; t += 2 * RING_ENC) {
        encode(t, fa, qa, 2);
        if (t + RING_ENC < count) encode(t + RING_ENC, fb, qb, 2);
    }
#elif ZS_RING_PF == 3
    // three items of register prefetch
    ObsPrefetch fa, fb, fc;
    zs_v2u qa, qb, qc;
    obs_prefetch_env(d, envc(t), OBS_OWN_ROWS, fa);
    obs_prefetch_env(d, envc(t + RING_ENC), obs_dirty(d, envc(t + RING_ENC)), fb);
    obs_prefetch_env(d, envc(t + 2 * RING_ENC), obs_dirty(d, envc(t + 2 * RING_ENC)), fc);
    qa = obs_dirty(d, envc(t + 3 * RING_ENC));
    qb = obs_dirty(d, envc(t + 4 * RING_ENC));
    qc = obs_dirty(d, envc(t + 5 * RING_ENC));
    for (; t < count; t += 3 * RING_ENC) {
        encode(t, fa, qa, 3);
        if (t + RING_ENC < count) encode(t + RING_ENC, fb, qb, 3);
        if (t + 2 * RING_ENC < count) encode(t + 2 * RING_ENC, fc, qc, 3);
    }
#else
    ObsPrefetch f;
    zs_v2u q0 = {0u, 0u};
    obs_prefetch(d, envc(t), envc(t + RING_ENC), obs_dirty(d, envc(t)), f);
    for (; t < count; t += RING_ENC) encode(t, f, q0, 1);
#endif
}

// ---------------------------------------------------------------------------
// k_obs_pbring: k_obs_ring's encoder / writer split on maps whose obstacle HP and dead-body rows are
// too large for the register prefetch (city128: 3689 obstacles, 512 dead-body words), with
// k_obs_gather's window-only fetches in the encoders.  An encoder wave takes an env in three load
// rounds: its entity table and dirty masks; its dead-body and obstacle-present words (a clean chunk
// from the shared zero / all-present rows) and the HP of its window cells' obstacles (a clean chunk from
// hp_init; the cells' static words from the workgroup's LDS tables, obs_stage_static4), the rounds
// software-pipelined so that an item's loads run while the previous one is encoded.  It encodes every
// agent's block into a ring slot (int32 staging for int64 output), and BRING_WRT writer waves stream the
// units out as 16-B stores, as in k_obs_ring.  Unit slots: as many as fit beside the tables and the
// encoder regions (us, at most 8 / PAIR; 5 for city128's 42-KB int64 envs).
// ---------------------------------------------------------------------------
// measured at C4 on one MI355X (2 runs each, profiles/r04_ab_c4_*.log): 9 / 3 159.5-159.9 us, 8 / 4 164.5,
// 8 / 3 170, 5 / 3 184-202, 12 / 3 (4 slots) 201; with the 63-lane cell walk 9 / 3 158.3-159.7, 10 / 2
// 153.6-155.0 (profiles/r04_ab_c4_enc.log)
#ifndef BRING_ENC
#define BRING_ENC 10
#endif
#ifndef BRING_WRT
#define BRING_WRT 2
#endif
#ifndef BRING_THR
#define BRING_THR RING_THR
#endif
#define BRING_D 8  // dead-body words per lane (DW <= 512)
#define BRING_O 2  // obstacle-present words per lane (OW <= 128, O <= 4096)
__host__ __device__ constexpr int bring_unit_bytes(int tsize, int nobs) {
    return obs_stage_slot_bytes(tsize, nobs * ring_pair(tsize, nobs));
}
__device__ __forceinline__ uint32_t chunk_of(uint32_t x, uint32_t m32) { return m32 ? __umulhi(x, m32) : x; }

// ---------------------------------------------------------------------------
// The encoding (round 5): a window cell costs its static word (obstacle, Box, objective bits and obstacle
// rank: the LDS tables of obs_stage_static4), the present bit of its obstacle, its dead-body bit and, for
// an obstacle, the HP its load round fetched (gym/observation.py:57-90: present obstacle > dead body >
// objective > empty), and then each present thing's lane (slot s on lane s) writes its code, life and
// weapon into every window it falls in (a thing takes precedence over everything on its cell).  The
// encoder's LDS region holds only the dead-body and present words.  (Round 6 removed k_obs_bring, the
// first form, which built per env a map of the thing on every window cell and looked it up per cell:
// 157.7 against 151.1 us at C4, profiles/r05f_ab_pbring.log.)
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int pbring_enc_bytes(int DW, int OW) { return ((DW * 4 + 15) / 16) * 16 + ((OW * 4 + 15) / 16) * 16; }
__host__ __device__ constexpr int pbring_fixed_bytes(int DW, int OW) { return 16 * DW + BRING_ENC * pbring_enc_bytes(DW, OW) + 128; }
__host__ __device__ constexpr int pbring_slots(int DW, int OW, int tsize, int nobs, int budget) {
    return (budget - pbring_fixed_bytes(DW, OW)) / bring_unit_bytes(tsize, nobs) < 8 / ring_pair(tsize, nobs)
               ? (budget - pbring_fixed_bytes(DW, OW)) / bring_unit_bytes(tsize, nobs)
               : 8 / ring_pair(tsize, nobs);
}

template <typename T, int NOBS>
__global__ void __launch_bounds__(64 * (BRING_ENC + BRING_WRT), 1) k_obs_pbring(Dev d, T* out, int env0, int env1, int us) {
    if (blockIdx.x == 0 && threadIdx.x == 0) step_tail(d);  // a zs_step's tail (Dev::tail_*)
    extern __shared__ __align__(16) uint8_t smem[];
    typedef typename obs_stage<T>::type S;
    constexpr int WW = 21, PLANE = WW * WW, PER = PLANE / 63, TS = (int)sizeof(T);
    static_assert(PLANE % 63 == 0, "63 lanes x PER rows of three");
    constexpr int PAIR = ring_pair(TS, NOBS), SLOT = obs_stage_slot_bytes(TS, NOBS * PAIR), BLK = NOBS * 3 * PLANE;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int encb = pbring_enc_bytes(d.DW, d.OW);
    lv4u* st4 = (lv4u*)smem;
    lu8* slots = (lu8*)(smem + 16 * d.DW + BRING_ENC * encb);
    ZS_LDS int* state = (ZS_LDS int*)(slots + us * SLOT);  // state[PAIR * slot + h], at most 8 words
    if (threadIdx.x < 8) state[threadIdx.x] = 0;
    obs_stage_static4(d, st4, threadIdx.x, blockDim.x);
    __syncthreads();
    const int G = gridDim.x, n_units = (env1 - env0 + PAIR - 1) / PAIR;
    const XcdDeal deal(blockIdx.x, G, n_units, BRING_WRT);
    const int ucount = deal.ucount;
    const int count = ucount ? PAIR * (ucount - 1) + min(PAIR, env1 - env0 - PAIR * deal.unit(ucount - 1)) : 0;
    auto unit_env = [&](int u) { return env0 + PAIR * deal.unit(u); };
    if (wave >= BRING_ENC) {  // writer
        for (int u = wave - BRING_ENC; u < ucount; u += BRING_WRT) {
            const int q = u % us, e = unit_env(u);
            const bool whole = PAIR * u + PAIR <= count;
            for (int h = 0; h < PAIR; h++)
                if (PAIR * u + h < count) ring_wait(&state[PAIR * q + h], 2 * u + 1);
            if (whole) obs_stage_flush<T, NOBS * PAIR, BRING_THR>(slots + q * SLOT, out + (size_t)e * BLK, lane);
            else obs_stage_flush<T, NOBS, BRING_THR>(slots + q * SLOT, out + (size_t)e * BLK, lane);
            for (int h = 0; h < PAIR; h++) ring_state_store(&state[PAIR * q + h], 2 * u + 2);
        }
        return;
    }
    // encoder
    lu32* idead = (lu32*)(smem + 16 * d.DW + wave * encb);
    lu32* iopres = (lu32*)(smem + 16 * d.DW + wave * encb + ((d.DW * 4 + 15) / 16) * 16);
    const int code_s = lane < d.A ? d.agent_codes[lane < d.A ? lane : 0] : (lane < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
    const int W = d.W, H = d.H, sl = lane < d.E ? lane : d.E - 1;
    // a lane's window cells: lane + 63 i, row lr + 3 i, column lq (lane 63 repeats lane 0's next cell)
    const int lr = lane / WW, lq = lane - lr * WW;
    auto item_env = [&](int t) { return unit_env(t / PAIR) + t % PAIR; };
    if (wave >= count) return;
    struct R1 {  // entity slot `lane`, dirty masks
        int32_t p, l, w, r;
        uint32_t hd, dd;
    };
    struct R23 {  // dead-body and present words; the HP of the window cells' obstacles
        uint32_t dv[BRING_D], ov[BRING_O];
        int32_t hv[NOBS][PER];
    };
    auto envc = [&](int t) { return item_env(t < count ? t : wave); };
    auto round1 = [&](int t, R1& r) {
        const int e = envc(t);
        r.p = d.pos[EIX(d, sl, e)];
        r.l = d.life[EIX(d, sl, e)];
        r.w = d.weapon[EIX(d, sl, e)];
        r.r = d.present[EIX(d, sl, e)];
        r.hd = d.hp_dirty[e];
        r.dd = d.dead_dirty[e];
    };
    // every load unconditional, addresses clamped; a window cell's obstacle index from the LDS tables (the
    // cell's rank among the map's obstacle cells, 0 where none: discarded by the encoding)
    auto round23 = [&](int t, const R1& r, R23& q) {
        const int e = envc(t);
        const uint32_t* dr = d.dead + (size_t)e * d.DW;
#pragma unroll
        for (int i = 0; i < BRING_D; i++) {
            const int w = min(lane + 64 * i, d.DW - 1);
            q.dv[i] = (((r.dd >> chunk_of((uint32_t)w, d.dead_chunk_m32)) & 1u) ? dr : d.dead_zero)[w];
        }
        const uint32_t* orow = r.hd ? d.obst_present + (size_t)e * d.OW : d.opres_full;
#pragma unroll
        for (int i = 0; i < BRING_O; i++) q.ov[i] = orow[min(lane + 64 * i, max(d.OW - 1, 0))];
        const int32_t* hrow = d.obst_hp + (size_t)e * d.O;
#pragma unroll
        for (int a = 0; a < NOBS; a++) {
            const int32_t ap = __builtin_amdgcn_readlane(r.p, a);
            const int ox = unpack_x(ap) - WW / 2, oy = unpack_y(ap) - WW / 2;
            const bool xin = (unsigned)(ox + lq) < (unsigned)W;
            const int c0 = (oy + lr) * W + ox + lq;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int y = oy + lr + 3 * i;
                const bool inb = xin && (unsigned)y < (unsigned)H;
                const int c = inb ? c0 + 3 * i * W : 0;
                const uint32_t bit = 1u << (c & 31);
                const zs_v4u sw = st4[c >> 5];
                const int o = (sw.x & bit) ? (int)(sw.w + __popc(sw.x & (bit - 1u))) : 0;
                q.hv[a][i] = (((r.hd >> chunk_of((uint32_t)o, d.hp_chunk_m32)) & 1u) ? hrow : d.hp_init)[o];
            }
        }
    };
    // the item's dead-body and present words into the wave's LDS region
    auto build = [&](const R23& q) {
#pragma unroll
        for (int i = 0; i < BRING_D; i++)
            if (lane + 64 * i < d.DW) idead[lane + 64 * i] = q.dv[i];
#pragma unroll
        for (int i = 0; i < BRING_O; i++)
            if (lane + 64 * i < d.OW) iopres[lane + 64 * i] = q.ov[i];
        wave_sync();
    };
    // every agent's block of item t into its unit's slot: the map pass, then the things over it
    auto encode = [&](int t, const R1& r, const R23& q) {
        const int u = t / PAIR, h = t % PAIR, e = item_env(t);
        const int qs = u % us;
        if (u >= us) ring_wait(&state[PAIR * qs + h], 2 * (u - us) + 2);
        wave_sync();
        ZS_LDS S* ot0 = (ZS_LDS S*)(slots + qs * SLOT) + (int)((uintptr_t)(out + (size_t)(e - h) * BLK) & 15) / TS + h * BLK;
#pragma unroll
        for (int a = 0; a < NOBS; a++) {
            const int32_t ap = __builtin_amdgcn_readlane(r.p, a);
            const int ox = unpack_x(ap) - WW / 2, oy = unpack_y(ap) - WW / 2;
            ZS_LDS S* ot = ot0 + a * 3 * PLANE;
            const bool xin = (unsigned)(ox + lq) < (unsigned)W;
            const int c0 = (oy + lr) * W + ox + lq;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int cell = lane + 63 * i;
                const int y = oy + lr + 3 * i;
                const bool inb = xin && (unsigned)y < (unsigned)H;
                const int c = inb ? c0 + 3 * i * W : 0;
                const uint32_t bit = 1u << (c & 31);
                const zs_v4u sw = st4[c >> 5];
                const uint32_t isob = (sw.x & bit) ? 1u : 0u;
                const int oi = isob ? (int)(sw.w + __popc(sw.x & (bit - 1u))) : 0;
                const bool obp = (isob & (iopres[oi >> 5] >> (oi & 31))) & 1u;
                int code = (idead[c >> 5] & bit) ? ZS_THING_DEADBODY : (sw.z & bit) ? ZS_THING_OBJECTIVE : ZS_THING_NONE;
                code = obp ? ((sw.y & bit) ? ZS_THING_BOX : ZS_THING_WALL) : code;
                code = inb ? code : ZS_THING_WALL;
                int life = obp ? q.hv[a][i] : 0;
                life = inb ? life : 200;
                if (cell < PLANE) {
                    ot[cell] = (S)code;
                    ot[PLANE + cell] = obs_val<S>(life);
                    ot[2 * PLANE + cell] = (S)0;
                }
            }
        }
        wave_sync();
        // the present things, slot s on lane s, over every agent's window
        if (lane < d.E && r.r) {
            const int x = unpack_x(r.p), y = unpack_y(r.p);
#pragma unroll
            for (int a = 0; a < NOBS; a++) {
                const int32_t ap = __builtin_amdgcn_readlane(r.p, a);
                const int dx = x - (unpack_x(ap) - WW / 2), dy = y - (unpack_y(ap) - WW / 2);
                if ((unsigned)dx < (unsigned)WW && (unsigned)dy < (unsigned)WW) {
                    ZS_LDS S* ot = ot0 + a * 3 * PLANE;
                    const int cc = dy * WW + dx;
                    ot[cc] = (S)code_s;
                    ot[PLANE + cc] = obs_val<S>(r.l);
                    ot[2 * PLANE + cc] = (S)r.w;
                }
            }
        }
        ring_state_store(&state[PAIR * qs + h], 2 * u + 1);
        wave_sync();  // the region is rebuilt for the next item
    };
    R1 ra, rb;
    R23 qa, qb;
    int t = wave;
    round1(t, ra);
    round1(t + BRING_ENC, rb);
    round23(t, ra, qa);
    // item t from set a while set b's later rounds run, then the roles swap
    auto step = [&](int t, R1& rx, R23& qx, R1& ry, R23& qy) {
        build(qx);
        round23(t + BRING_ENC, ry, qy);
        const R1 cur = rx;  // the item's entity row (its things and agent positions), then the row two items on
        round1(t + 2 * BRING_ENC, rx);
        encode(t, cur, qx);
    };
    for (; t < count; t += 2 * BRING_ENC) {
        step(t, ra, qa, rb, qb);
        if (t + BRING_ENC < count) step(t + BRING_ENC, rb, qb, ra, qa);
    }
}
