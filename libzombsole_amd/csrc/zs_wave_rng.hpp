// zs_wave_rng.hpp — one env's CPython MT19937 stream consumed by a whole wave.
//
// Long runs of draws (the Fisher-Yates passes of World.spawn_in_random, core.py:40-66, whose
// candidate lists reach thousands of cells) are resolved 64 words at a time: the stream is held
// one word per lane, every _randbelow (random.py:239-249) rejection chain is walked with ballots,
// and a block of 624 words that runs out is twisted cooperatively.  Two stream holders:
//   WaveRng (k_reset): the env's ring staged in LDS for the whole reset, flushed at the end;
//   GRng    (k_tick's cooperative respawn): the ring read from HBM (L1-bypassing loads) and
//           twisted in registers (no LDS: the tick's LDS is its occupancy).
#pragma once
#include "zs_device.hpp"

#define WR_Q 4               // words per lane held in registers
#define WR_BLOCK (64 * WR_Q)  // words per register block

struct WaveRng {
    uint32_t st;          // ring state of the register block's word 0 (uniform)
    int pos;              // next unconsumed word within the block (uniform, 0..WR_BLOCK)
    uint32_t word[WR_Q];  // word[q] = tempered stream word q*64 + lane of the block
    uint32_t* ring;       // the env's ring in HBM (read once at the start, dirty slots written at the end)
    lu32* lr;             // its LDS copy, 2 x 624 words: every draw and twist of the reset works here
    int dirty;            // bit s: LDS slot s was twisted and must be written back
};

// stage the env's ring into LDS: both slots, whatever the stream state (the slot not yet twisted holds
// stale words that nothing reads before wave_twist rewrites them), so the loads do not wait for the
// state word.  wave_rng_fetch issues the 20 loads per lane, wave_rng_put stores them: a caller issues
// its other loads in between, and the round trips overlap.
#define WR_STAGE_K ((2 * ZS_MT_N + 63) / 64)
__device__ __forceinline__ void wave_rng_fetch(const WaveRng& r, uint32_t (&v)[WR_STAGE_K]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < WR_STAGE_K; u++) v[u] = r.ring[min(lane + 64 * u, 2 * ZS_MT_N - 1)];
}
__device__ __forceinline__ void wave_rng_put(WaveRng& r, const uint32_t (&v)[WR_STAGE_K]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < WR_STAGE_K; u++)
        if (lane + 64 * u < 2 * ZS_MT_N) r.lr[lane + 64 * u] = v[u];
    r.dirty = 0;
    wave_sync();
}
__device__ __forceinline__ void wave_rng_stage(WaveRng& r) {
    uint32_t v[WR_STAGE_K];
    wave_rng_fetch(r, v);
    wave_rng_put(r, v);
}

// next block of the stream (LDS slot ^ 1) from the current one (_randommodule.c genrand_uint32's
// twist), cooperatively in three dependency phases
__device__ __forceinline__ void wave_twist(WaveRng& r, uint32_t slot) {
    const int lane = threadIdx.x & 63;
    const lu32* src = r.lr + slot * ZS_MT_N;
    lu32* nw = r.lr + (slot ^ 1u) * ZS_MT_N;
    for (int k = lane; k < ZS_MT_N - ZS_MT_M; k += 64) nw[k] = mt_f(src[k], src[k + 1], src[k + ZS_MT_M]);
    wave_sync();
    for (int k = (ZS_MT_N - ZS_MT_M) + lane; k < 2 * (ZS_MT_N - ZS_MT_M); k += 64)
        nw[k] = mt_f(src[k], src[k + 1], nw[k + ZS_MT_M - ZS_MT_N]);
    wave_sync();
    for (int k = 2 * (ZS_MT_N - ZS_MT_M) + lane; k < ZS_MT_N; k += 64)
        nw[k] = mt_f(src[k], k + 1 < ZS_MT_N ? src[k + 1] : nw[0], nw[k + ZS_MT_M - ZS_MT_N]);
    wave_sync();
    r.dirty |= 1 << (slot ^ 1u);
}

// write the twisted slots back to the env's ring in HBM (no wait: the next reader is a later launch)
__device__ __forceinline__ void wave_rng_flush(const WaveRng& r) {
    const int lane = threadIdx.x & 63;
    for (int sl = 0; sl < 2; sl++)
        if ((r.dirty >> sl) & 1)
            for (int k = lane; k < ZS_MT_N; k += 64) r.ring[sl * ZS_MT_N + k] = r.lr[sl * ZS_MT_N + k];
}

// load the WR_BLOCK words that start at ring state st (twisting the next block first if needed)
__device__ __forceinline__ void rng_block_load(WaveRng& r, uint32_t st) {
    uint32_t off = st & 1023u, slot = (st >> 10) & 1u, ready = (st >> 11) & 1u;
    if (off >= ZS_MT_N) {
        if (!ready) wave_twist(r, slot);
        slot ^= 1u;
        off = 0;
        ready = 0;
    }
    if (off + WR_BLOCK > ZS_MT_N && !ready) {
        wave_twist(r, slot);
        ready = 1;
    }
#pragma unroll
    for (int q = 0; q < WR_Q; q++) {
        uint32_t p = off + q * 64 + (threadIdx.x & 63);
        r.word[q] = mt_temper(p < ZS_MT_N ? r.lr[slot * ZS_MT_N + p] : r.lr[(slot ^ 1u) * ZS_MT_N + p - ZS_MT_N]);
    }
    r.st = st_pack(off, slot, ready);
    r.pos = 0;
}

template <class R>
__device__ __forceinline__ uint32_t wr_sub(const R& r, int q) {
    return q == 0 ? r.word[0] : q == 1 ? r.word[1] : q == 2 ? r.word[2] : r.word[3];
}

// `count` consecutive draws _randbelow(b_t), b_t = n - t * dstep (dstep 0: a fixed bound; 1: the
// decreasing bounds of a Fisher-Yates pass), all in wave-uniform control flow.  Draw t consumes
// words until one word w gives (w >> (32 - bitlen(b_t))) < b_t (random.py:239-249).
//
// One round per 64-word sub-block: the word of lane l serves draw t_l = done + (l - start) - H_l,
// H_l = the rejected words of this round before lane l, a sequential definition.  It is solved as a
// fixed point: from H = 0, every lane evaluates its word, one ballot gives the rejections, prefix
// counts give the next H; the first lane is exact after one pass and lane start + j after j + 1, so
// the iteration ends, and a pass that leaves the ballot unchanged satisfies the recurrence at every
// lane, i.e. is its solution.  A change of H moves a lane's bound by one (dstep 1) or not at all
// (dstep 0), which flips its outcome only at a bit-length or threshold edge: usually two passes.
// Every accepted lane then hands its draw's value to put(t, value) for t < krec.  Advances r past
// the consumed words.
template <class R, class Put>
__device__ __forceinline__ void wave_draws(R& r, int n, int dstep, int count, int krec, Put put) {
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    int done = 0;
    while (done < count) {
        if (r.pos >= WR_BLOCK) rng_block_load(r, st_advance(r.st, WR_BLOCK));
        const int q = r.pos >> 6, base = q << 6, start = r.pos - base;
        const uint32_t w = wr_sub(r, q);
        const int idx = lane - start;
        unsigned long long rej = 0ull, prev;
        int t;
        bool lv, rj;
        do {
            prev = rej;
            t = done + idx - __popcll(rej & below);
            lv = idx >= 0 && t < count;
            const int b = n - t * dstep;
            const int kk = 32 - __clz(max(b, 1));
            rj = lv && (w >> (32 - kk)) >= (uint32_t)b;
            rej = __ballot(rj);
        } while (rej != prev);
        // live lanes (t < count) are a prefix of [start, 64): t never decreases along the lanes
        const unsigned long long live = __ballot(lv);
        if (lv && !rj && t < krec) {
            const int b = n - t * dstep;
            put(t, w >> (32 - (32 - __clz(b))));
        }
        done += __popcll(live) - __popcll(rej);
        r.pos = base + 64 - __clzll((long long)live);
    }
    wave_sync();
}

