// engine.hip — MI355X-native batched zombsole step engine (gfx950) and its C ABI.
//
// A step (zs_step) is: k_reset (zs_reset.hpp, one wave per env that ended at the previous step, on
// a side stream concurrent with the tick, or fused with it into k_step), k_tick (zs_tick.hpp, 64/G
// envs per wave with G lanes per env and the env's hot state in LDS), k_respawn (deferred zombie
// respawns, one wave per env) and the observation kernel (zs_obs.hpp: k_obs_ring / k_obs_pipe
// persistent store streams, k_obs_gather for large maps, k_obs in general).  zs_step_graph replays
// a step as a hipGraph.  k_seed / k_gen_actions / k_get_state / k_set_state are the small helpers
// behind the ABI.
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

#include "zs_launch.hpp"
#include "zs_reset.hpp"
#include "zs_obs.hpp"

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
// bench / parity action stream (libzombsole_amd/actions.py; policy_action in zs_device.hpp)
// ---------------------------------------------------------------------------
// one thread per (env, agent): its triple
__global__ void k_gen_actions(Dev d, uint64_t step, int n_discrete, int32_t* act) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.N * d.A) return;
    const int e = i / d.A;
    const int id = policy_id(d.seeds[e], step, n_discrete, i - e * d.A);
    act[(size_t)i * 3 + 0] = c_discrete[id][0];
    act[(size_t)i * 3 + 1] = c_discrete[id][1];
    act[(size_t)i * 3 + 2] = c_discrete[id][2];
}

// The same policy for the step number in device memory (zs_step_graph with the reset work on a side
// stream: launched after the reset fork, it gives the reset work a head start on the tick)
__global__ void k_gen_actions_ctr(Dev d, const uint64_t* ctr, int n_discrete, int32_t* act) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.N * d.A) return;
    const int e = i / d.A;
    const int id = policy_id(d.seeds[e], ctr[0], n_discrete, i - e * d.A);
    act[(size_t)i * 3 + 0] = c_discrete[id][0];
    act[(size_t)i * 3 + 1] = c_discrete[id][1];
    act[(size_t)i * 3 + 2] = c_discrete[id][2];
}

// the step's tail when no observation launch ends the step (observations written by the step launch)
__global__ void k_tail(Dev d) {
    if (threadIdx.x == 0) step_tail(d);
}

// ---------------------------------------------------------------------------
// state views (one env, one thread; test pokes)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int state_words(const Dev& d) {
    return ZS_STATE_HEADER + ZS_STATE_ENTITY_WORDS * d.E + d.E + 2 * d.O + 2 * d.A + d.DW;
}

// env e's state record (layout: include/zombsole_mi355x.h), written by threads tid = 0..nt-1 of one workgroup
// (every thread of the workgroup calls it)
__device__ void state_record(const Dev& d, int e, int32_t* b, int tid, int nt) {
    const int N = d.N, E = d.E;
    __shared__ int nz;  // present zombies
    if (tid == 0) nz = 0;
    __syncthreads();
    for (int s = d.A + d.P + tid; s < E; s += nt)
        if (d.present[EIX(d, s, e)]) atomicAdd(&nz, 1);
    __syncthreads();
    if (tid == 0) {
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
        b[11] = nz;
        b[12] = d.scal[S_SERIAL * N + e];
        b[13] = b[14] = b[15] = 0;
    }
    int32_t* r = b + ZS_STATE_HEADER;
    for (int s = tid; s < E; s += nt) {
        int32_t* q = r + s * ZS_STATE_ENTITY_WORDS;
        int32_t p = d.pos[EIX(d, s, e)];
        q[0] = s < d.A ? ZS_THING_AGENT : (s < d.A + d.P ? ZS_THING_PLAYER : ZS_THING_ZOMBIE);
        q[1] = d.present[EIX(d, s, e)];
        q[2] = unpack_x(p);
        q[3] = unpack_y(p);
        q[4] = d.life[EIX(d, s, e)];
        q[5] = d.weapon[EIX(d, s, e)];
        q[6] = s < d.A ? s : (s < d.A + d.P ? s - d.A : 0);
        q[7] = (int32_t)d.serial[EIX(d, s, e)];
    }
    r += ZS_STATE_ENTITY_WORDS * E;
    for (int s = tid; s < E; s += nt) r[s] = d.order[EIX(d, s, e)];
    r += E;
    for (int o = tid; o < d.O; o += nt) r[o] = d.obst_hp[(size_t)e * d.O + o];
    r += d.O;
    for (int o = tid; o < d.O; o += nt) r[o] = (d.obst_present[(size_t)e * d.OW + (o >> 5)] >> (o & 31)) & 1u;
    r += d.O;
    for (int a = tid; a < d.A; a += nt) r[a] = d.prev_life[(size_t)a * N + e];
    r += d.A;
    for (int a = tid; a < d.A; a += nt) r[a] = d.listed[(size_t)a * N + e];
    r += d.A;
    for (int w = tid; w < d.DW; w += nt) r[w] = (int32_t)d.dead[(size_t)e * d.DW + w];
}

__global__ void k_get_state(Dev d, int e, int32_t* buf) { state_record(d, e, buf, threadIdx.x, blockDim.x); }

// ---------------------------------------------------------------------------
// the drop-ins' per-call path (zs_host_step / zs_host_reset / zs_host_observe): one workgroup per env
// ---------------------------------------------------------------------------
// the process-global `random` state moved in (rings[e]: the getstate() block and its successor, st[e])
// (host memory read in place: one round of 16-B loads, 1 248 words = 312 per env)
__global__ void k_host_unpack(Dev d, const uint32_t* rings, const uint32_t* st) {
    const int e = blockIdx.x, t = threadIdx.x;
    static_assert(ZS_RING_WORDS % 4 == 0, "16-B copies");
    const uint4* src = (const uint4*)(rings + (size_t)e * ZS_RING_WORDS);
    uint4* dst = (uint4*)(d.ring + (size_t)e * ZS_RING_WORDS);
    const int n4 = ZS_RING_WORDS / 4;  // 312: two per thread at most (blockDim 256)
    uint4 a = t < n4 ? src[t] : uint4{}, b = t + 256 < n4 ? src[t + 256] : uint4{};
    const uint32_t sv = t == 0 ? st[e] : 0u;
    if (t < n4) dst[t] = a;
    if (t + 256 < n4) dst[t + 256] = b;
    if (t == 0) d.rngst[e] = sv;
}

// Word offsets of a host record's sections (ZS_HOST_* in include/zombsole_mi355x.h, zs_host_layout)
struct HostLayout {
    int words, rew, alog, dlog, state, obs, obs_bytes, R;
};

// everything a call returns to the host, for env e: outputs, RNG stream, logs, state record, observation
__global__ void k_host_pack(Dev d, HostLayout L, const uint8_t* obs, const double* rew, const uint8_t* done,
                            const uint8_t* trunc, const uint8_t* rst, int* err, int32_t* rec) {
    const int e = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    int32_t* r = rec + (size_t)e * L.words;
    const uint32_t st = d.rngst[e];
    if (tid == 0) {
        r[ZS_HOST_FLAGS] = (done[e] ? 1 : 0) | (trunc[e] ? 2 : 0) | (rst && rst[e] ? 4 : 0);
        r[ZS_HOST_ERR] = *err;
        *err = 0;  // the next call's error word starts clear (no memset launch)
        r[ZS_HOST_ALOG_N] = d.alog ? d.alog_n[e] : 0;
        r[ZS_HOST_DLOG_N] = d.dlog ? d.dlog_n[e] : 0;
        r[ZS_HOST_RNG + ZS_MT_N] = (int32_t)(st & 1023u);
    }
    const uint32_t* blk = d.ring + (size_t)e * ZS_RING_WORDS + ((st >> 10) & 1u) * ZS_MT_N;
    for (int k = tid; k < ZS_MT_N; k += nt) r[ZS_HOST_RNG + k] = (int32_t)blk[k];
    const int32_t* rw = (const int32_t*)(rew + (size_t)e * L.R);
    for (int k = tid; k < 2 * L.R; k += nt) r[L.rew + k] = rw[k];
    if (d.alog)
        for (int k = tid; k < 2 * d.E; k += nt) r[L.alog + k] = d.alog[(size_t)e * d.E * 2 + k];
    if (d.dlog)
        for (int k = tid; k < 5 * d.E; k += nt) r[L.dlog + k] = d.dlog[(size_t)e * d.E * 5 + k];
    state_record(d, e, r + L.state, tid, nt);
    // the observation: 16-B copies when the env's block allows (L.obs is 16-B aligned), else 2-B ones
    const uint8_t* src = obs + (size_t)e * L.obs_bytes;
    uint8_t* dst = (uint8_t*)(r + L.obs);
    if (L.obs_bytes % 16 == 0 && ((size_t)e * L.obs_bytes) % 16 == 0 && (L.words % 4) == 0) {
        for (int k = tid; k < L.obs_bytes / 16; k += nt) ((uint4*)dst)[k] = ((const uint4*)src)[k];
    } else {
        for (int k = tid; k < L.obs_bytes / 2; k += nt) ((uint16_t*)dst)[k] = ((const uint16_t*)src)[k];
    }
}

__global__ void k_set_state(Dev d, int e, const int32_t* buf, int* err) {
    if (threadIdx.x != 0) return;
    const int N = d.N, E = d.E;
    const int32_t* b = buf;
    // needs_reset (b[5]) is the engine's own: pending resets are its work lists (an env on a list with
    // the flag cleared would be reset and ticked by one call, one off the lists with the flag set would
    // report a reset without a rebuild), so a record that disagrees is refused, nothing written
    if (b[5] != d.scal[S_NEEDRESET * N + e]) {
        *err = ZS_EINVAL;
        return;
    }
    d.scal[S_T * N + e] = b[0];
    d.scal[S_DEATHS * N + e] = b[1];
    d.scal[S_ZD * N + e] = b[2];
    d.scal[S_EPSTEPS * N + e] = b[3];
    d.scal[S_NORDER * N + e] = b[4];
    d.scal[S_PREVZD * N + e] = b[10];
    d.scal[S_SERIAL * N + e] = b[12];
    const int32_t* r = b + ZS_STATE_HEADER;
    for (int s = 0; s < E; s++, r += ZS_STATE_ENTITY_WORDS) {
        d.present[EIX(d, s, e)] = (uint8_t)r[1];
        d.pos[EIX(d, s, e)] = pack_xy(r[2], r[3]);
        d.life[EIX(d, s, e)] = r[4];
        d.weapon[EIX(d, s, e)] = (uint8_t)r[5];
        d.serial[EIX(d, s, e)] = (uint32_t)r[7];
    }
    for (int s = 0; s < E; s++) d.order[EIX(d, s, e)] = (uint8_t)*r++;
    int any_nonpos = 0;
    for (int o = 0; o < d.O; o++) {
        int v = *r++;
        d.obst_hp[(size_t)e * d.O + o] = hp_store_value(d, v);
        d.hp_dirty[e] = 0xffffffffu;
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
    d.dead_dirty[e] = 0xffffffffu;
}

__global__ void k_init_pending(Dev d, int* list, int* count) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e == 0) {
        count[0] = d.N;
        count[1] = 0;
    }
    if (e >= d.N) return;
    list[e] = e;
    d.scal[S_NEEDRESET * d.N + e] = 1;
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

// the observation launcher of the handle's output dtype (k_obs_t.hip)
static hipError_t obs_launch(int dtype, const ObsLaunch& o, hipStream_t s, const Dev& d) {
    return dtype == ZS_DTYPE_I64 ? launch_obs_i64(o, s, d) : dtype == ZS_DTYPE_I32 ? launch_obs_i32(o, s, d) : launch_obs_i16(o, s, d);
}
static hipError_t obs_attr(int dtype, int kind, int nobs, int patched, int bytes) {
    return dtype == ZS_DTYPE_I64   ? obs_lds_attr_i64(kind, nobs, patched, bytes)
           : dtype == ZS_DTYPE_I32 ? obs_lds_attr_i32(kind, nobs, patched, bytes)
                                   : obs_lds_attr_i16(kind, nobs, patched, bytes);
}

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t _e = (x);                                                                   \
        if (_e != hipSuccess) return fail(ZS_EHIP, std::string(#x ": ") + hipGetErrorString(_e)); \
    } while (0)

struct zs_handle {
    zs_config cfg;
    zs_launch ov;   // launch overrides (zs_config.launch, zeroed when NULL)
    int device;
    Dev d;
    int G;          // lanes per env in k_tick
    int tick_waves = ZS_STEP_WAVES;  // k_tick's register budget (waves per SIMD it is compiled for)
    size_t lds;     // k_tick dynamic LDS bytes
    ObsLayout obs_l;  // k_obs per-wave LDS image
    int obs_wpg;      // k_obs waves (envs) per workgroup
    int obs_pipe = 0;      // k_obs_pipe<NOBS> usable (NOBS = 1, 2, 4), else 0
    int obs_ring = 0;      // k_obs_ring: encoder and writer waves through an LDS ring (zs_launch.obs_ring)
    size_t obs_ring_bytes = 0;
    int obs_bring = 0;     // k_obs_pbring: its unit slots (0: not used)
    size_t obs_bring_bytes = 0;
    int obs_patch = 0;     // k_obs_pipe's walk with the padded-table encoder and the staged flush (k_obs_patch)
    size_t obs_patch_bytes = 0;
    int obs_patch_wgs = 2;  // its workgroups (PATCH_WPG waves) per CU
    int obs_gather = 0;    // else k_obs_gather<NOBS> usable (NOBS = 1, 2, 4), else 0 (k_obs)
    int obs_gather_stat = 0;    // k_obs_gather reads the static words from LDS tables (zs_launch.obs_gather_stat)
    ObsLayout obs_gl;      // its per-wave image
    // zs_step_graph: one captured hipGraph per autoreset-list parity (the step alternates the two
    // pending-reset lists), replayed on the caller's stream; keyed by the caller's buffers
    // a few buffer sets cached (a caller alternating double-buffered outputs, vector.StepGather)
    struct GraphSet {
        hipGraphExec_t g[2] = {nullptr, nullptr};  // per pending-list parity
        const void* key[9] = {};
        uint64_t used = 0;
    };
    static const int kGraphSets = 4;
    GraphSet gsets[kGraphSets];
    uint64_t gclock = 0;
    uint64_t* d_gstep = nullptr;  // [0] policy step counter (the step's policy reads it, the step's tail advances it)
    int graph_pol = 0;            // zs_step_graph is capturing a step with this policy (n_discrete), else 0
    int obs_pipe_wgs = 8;  // k_obs_pipe workgroups per CU
    // next-step reset work on a side stream, concurrent with the tick (the two touch disjoint envs);
    // the caller's stream joins it before the observations
    int reset_side = 0;
    hipStream_t s_reset = nullptr;
    hipEvent_t ev_rfork = nullptr, ev_rjoin = nullptr;
    int state_words;
    std::vector<void*> allocs;
    int32_t* d_state;
    uint64_t* d_seedbuf;
    int* d_err;
    // next-step autoreset work lists: k_tick appends to list[1-par], k_reset drains list[par]
    int* d_rlist[2];
    int* d_rcount;  // [2]
    int rpar = 0;
    size_t reset_lds = 0;
    int fused = 0;  // zs_step runs reset work and the tick in one launch (k_step)
    int resident = 0;  // step-launch workgroups resident per CU (layout choice)
    int want = 0;      // workgroups per CU the launch has (capped at 32)
    // the drop-ins' per-call path (zs_host_*), set up by its first call: one pinned, device-mapped input
    // block (actions, then the `random` state as rings + st words) the kernels read in place, one pinned,
    // device-mapped record block k_host_pack writes in place, one synchronisation per call
    HostLayout hl{};
    int32_t* h_hin = nullptr;   // pinned host memory ...
    int32_t* d_hin = nullptr;   // ... and its device address
    int32_t* h_hrec = nullptr;
    int32_t* d_hrec = nullptr;
    uint8_t* d_hobs = nullptr;
    double* d_hrew = nullptr;
    uint8_t* d_hflags = nullptr;  // done [N], trunc [N], listed [N][A], reset [N]
    // diagnostics: HIP events bracketing every k_tick / k_obs launch on its stream
    int prof = 0;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, int>> ev_tick, ev_obs, ev_reset, ev_respawn;  // (start, end) indices into ev_pool
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
    if (h->h_hin) (void)hipHostFree(h->h_hin);
    if (h->h_hrec) (void)hipHostFree(h->h_hrec);
    h->h_hin = h->h_hrec = nullptr;
    if (h->ev_rfork) (void)hipEventDestroy(h->ev_rfork);
    if (h->ev_rjoin) (void)hipEventDestroy(h->ev_rjoin);
    h->ev_rfork = h->ev_rjoin = nullptr;
    if (h->s_reset) (void)hipStreamDestroy(h->s_reset);
    h->s_reset = nullptr;
    for (auto& gs : h->gsets)
        for (hipGraphExec_t& g : gs.g)
            if (g) {
                (void)hipGraphExecDestroy(g);
                g = nullptr;
            }
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

// Layout of the step launch.  Workgroups of the launch resident at once on the 256 CUs decide how
// much LDS one may take: among the layouts that fit 64 KiB, take the one with the most resident
// workgroups (at most 32 one-wave workgroups per CU), then the largest optional LDS copies (RNG
// window beyond 64 words, spawn candidates, spawn lists).  A fused launch (reset work + tick in
// one) allocates max(tick image, reset image) for every workgroup.
// reset-work workgroups of a fused step launch (zs_launch.reset_wgs overrides)
static int reset_wgs(const zs_handle* h) { return h->ov.reset_wgs > 0 ? h->ov.reset_wgs : 256; }

static int choose_layout(zs_handle* h, int want_g, bool fused, int obs_bytes) {
    Dev& d = h->d;
    const int kMax = 64 * 1024;
    // A launch of many resident rounds is bound by the envs it keeps in flight per CU (k_tick at C3:
    // 19 -> 15 resident workgroups of G = 8 took the launch from 121 to 153 us), a one-round launch by
    // the latency of one workgroup.  Measured on one MI355X: G = 8 beats 16 when G = 16 needs more
    // than two rounds (C3, 65536 envs, E = 12: 121 vs 140 us), G = 16 beats 8 at 8192 and 16384 envs
    // and at C5 (E = 24); G = 32 beats 16 at C4 (E = 54: the decisions spread over more lanes).
    // one-wave workgroups per CU the register budget admits (k_step's or k_tick's)
    const int wave_cap = 4 * (fused ? ZS_FUSED_WAVES : ZS_STEP_WAVES);
    int g0 = want_g > 0 ? want_g : (d.E > 32 ? 32 : 16);
    if (want_g <= 0 && d.E <= 16 && (long)d.N > 2L * wave_cap * 256 * (64 / 16)) g0 = 8;
    int cand_full = (d.W * d.H <= 65535) ? d.ncand : 0;
    // RNG window: a plain step draws about 1.5 words per actor (shuffle) plus one per attack or heal
    // in range; a window that runs dry sends the leader to HBM.  Measured with the oracle (uniform
    // Discrete(7) agents): C3 (E = 12) mean 12, p99 26, max 37 words; C5 (E = 24) mean 23, p99 46,
    // max 63; C4 (E = 54) median 82.  2E + 8 rounded up to a power of two covers them.
    int rw_need = 32;
    while (rw_need < 512 && rw_need < 2 * d.E + 8) rw_need *= 2;
    if (h->ov.rw_need > 0) rw_need = std::max(32, std::min(512, (int)h->ov.rw_need));
    int lists = (d.nps + d.nzs <= 4096) ? d.nps + d.nzs : 0;
    for (int G = g0; G <= 64; G *= 2) {
        int ne = 64 / G;
        int wgs = (d.N + ne - 1) / ne + (fused ? std::min(d.N, reset_wgs(h)) : 0);
        int want = h->ov.lds_budget < 0 ? 1 : std::min(32, std::max(1, (wgs + 255) / 256));
        int best_res = -1;
        for (int pass = 0; pass < 2 && best_res < 0; pass++)  // windows below the need only if nothing else fits
        for (int cand : {cand_full, 0})
            for (int lst : {lists, 0})
                for (int rw : {512, 256, 128, 64, 32}) {
                    if (pass == 0 && rw < rw_need) continue;
                    int bytes = tick_layout(ne, d.E, d.DW, rw, cand, lst, d.A, obs_bytes).bytes;
                    if (fused) bytes = std::max(bytes, reset_lds_bytes(d.E, d.DW, d.ncand, lst, obs_bytes));
                    if (bytes > kMax) continue;
                    int res = std::min(std::min(want, wave_cap), 160 * 1024 / bytes);
                    h->want = want;
                    if (res > best_res) {
                        best_res = res;
                        h->G = G;
                        d.rw_cap = rw;
                        d.rw_step = std::min(rw, rw_need);
                        d.cand_cap = cand;
                        d.lists_cap = lst;
                        h->lds = bytes;
                        h->resident = res;
                    }
                }
        if (best_res > 0) return ZS_OK;
    }
    return fail(ZS_EINVAL, "entity table / map too large for the LDS image of one env");
}

extern "C" int zs_create(const zs_config* cfg, int device, zs_handle** out) {
    if (!cfg || !out) return fail(ZS_EINVAL, "null argument");
    int rc = validate(cfg);
    if (rc) return rc;
    HIPCHK(hipSetDevice(device));
    zs_handle* h = new zs_handle();
    h->cfg = *cfg;
    memset(&h->ov, 0, sizeof(h->ov));
    if (cfg->launch) h->ov = *cfg->launch;
    h->cfg.launch = nullptr;
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
    // zombie respawn as wave work after the tick (k_respawn) when its shuffle is long: the tick's
    // leader would draw one word per candidate serially.  zs_launch.defer_respawn forces either.
    {
        const int cands = m.n_zombie_spawns ? m.n_zombie_spawns : d.W * d.H;
        const int dr = h->ov.defer_respawn;
        d.defer_respawn = d.minimum_zombies > 0 && (dr ? dr > 0 : cands > 64);
    }

    // the shuffle and execution of a tick's actions by the env's lanes (zs_tick.hpp grp_execute) instead of
    // its leader lane alone; zs_launch.par_exec = -1 keeps the leader's serial loop (A/B, parity tests)
    d.par_exec = h->ov.par_exec >= 0;
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
    std::vector<uint32_t> obstbits(d.DW, 0);
    for (int i = 0; i < d.O; i++) {
        int cell = m.obstacle_xy[2 * i + 1] * d.W + m.obstacle_xy[2 * i];
        obstbits[cell >> 5] |= 1u << (cell & 31);
    }
    // the observation store loop finds an obstacle's index as the rank of its cell among obstacle
    // cells (zs_obs.hpp), valid when the obstacles are in row-major order (every map-file parse)
    bool rank_order = true;
    for (int i = 1; i < d.O; i++)
        if (m.obstacle_xy[2 * i + 1] * d.W + m.obstacle_xy[2 * i] <=
            m.obstacle_xy[2 * i - 1] * d.W + m.obstacle_xy[2 * i - 2])
            rank_order = false;
    std::vector<uint32_t> boxbits(d.DW, 0);
    for (int i = 0; i < d.O; i++)
        if (m.obstacle_kind[i] == ZS_THING_BOX) {
            int cell = m.obstacle_xy[2 * i + 1] * d.W + m.obstacle_xy[2 * i];
            boxbits[cell >> 5] |= 1u << (cell & 31);
        }
    std::vector<int32_t> oprefix(d.DW, 0);
    for (int w = 1; w < d.DW; w++) oprefix[w] = oprefix[w - 1] + __builtin_popcount(obstbits[w - 1]);
    std::vector<uint32_t> objbits(d.DW, 0);
    std::vector<int32_t> scell((size_t)d.W * d.H, 0);  // k_obs static per-cell word (zs_obs.hpp)
    for (int i = 0; i < m.n_objectives; i++) {
        int cell = m.objective_xy[2 * i + 1] * d.W + m.objective_xy[2 * i];
        objbits[cell >> 5] |= 1u << (cell & 31);
        scell[cell] |= (int32_t)SC_OBJ_BIT;
    }
    for (int i = 0; i < d.O; i++) {
        int cell = m.obstacle_xy[2 * i + 1] * d.W + m.obstacle_xy[2 * i];
        scell[cell] |= (int32_t)((uint32_t)(i + 1) | ((uint32_t)m.obstacle_kind[i] << SC_KIND_SHIFT));
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
    uint32_t *p_objbits, *p_obstbits, *p_boxbits;
    int32_t *p_scell, *p_oprefix;
    int32_t *p_oxy, *p_ps, *p_zs, *p_aw, *p_ac, *p_bt;
    uint8_t* p_okind;
    TRY(dupload(h, &p_cellmap, cellmap));
    TRY(dupload(h, &p_objbits, objbits));
    TRY(dupload(h, &p_obstbits, obstbits));
    TRY(dupload(h, &p_scell, scell));
    TRY(dupload(h, &p_boxbits, boxbits));
    TRY(dupload(h, &p_oprefix, oprefix));
    TRY(dupload(h, &p_oxy, oxy));
    TRY(dupload(h, &p_okind, okind));
    TRY(dupload(h, &p_ps, ps));
    TRY(dupload(h, &p_zs, zs));
    TRY(dupload(h, &p_aw, aw));
    TRY(dupload(h, &p_ac, ac));
    TRY(dupload(h, &p_bt, bt));
    {
        // k_obs_patch's tables (zs_obs.hpp): the map padded by half a registered window (21) on every
        // side, each cell the code / life it shows with no thing on it, no body, every obstacle present
        // at MAX_LIFE (out of bounds: Wall 200, gym/observation.py:69-76); per obstacle x | y << 12 |
        // box << 24 | objective-under << 25
        const int half = 10, pw = d.W + 2 * half, ph = d.H + 2 * half;
        std::vector<uint16_t> pad((((size_t)pw * ph + 7) / 8) * 8, 0);
        for (int y = -half; y < d.H + half; y++)
            for (int x = -half; x < d.W + half; x++) {
                uint16_t v = (uint16_t)(ZS_THING_WALL | (200 << 8));
                if (x >= 0 && y >= 0 && x < d.W && y < d.H) {
                    const int c = y * d.W + x;
                    const bool obj = (objbits[c >> 5] >> (c & 31)) & 1u;
                    const int oi = cellmap[c];
                    if (oi >= 0)
                        v = okind[oi] == ZS_THING_BOX ? (uint16_t)(ZS_THING_BOX | (10 << 8)) : (uint16_t)(ZS_THING_WALL | (200 << 8));
                    else
                        v = obj ? ZS_THING_OBJECTIVE : ZS_THING_NONE;
                    if (oi >= 0 && obj) v |= OPAD_OBJ;
                }
                pad[(size_t)(y + half) * pw + x + half] = v;
            }
        std::vector<uint32_t> opk(std::max(d.O, 1), 0u);
        for (int i = 0; i < d.O; i++) {
            const int x = m.obstacle_xy[2 * i], y = m.obstacle_xy[2 * i + 1], c = y * d.W + x;
            opk[i] = (uint32_t)(x & 0xfff) | ((uint32_t)(y & 0xfff) << 12) | ((okind[i] == ZS_THING_BOX ? 1u : 0u) << 24) |
                     (((objbits[c >> 5] >> (c & 31)) & 1u) << 25);
        }
        uint16_t* p_pad;
        uint32_t* p_opk;
        TRY(dupload(h, &p_pad, pad));
        TRY(dupload(h, &p_opk, opk));
        d.opad = p_pad;
        d.opad_w = pw;
        d.opad_n = pw * ph;
        d.opk = p_opk;
    }
    d.cellmap = p_cellmap;
    d.objbits = p_objbits;
    d.obstbits = p_obstbits;
    d.scell = p_scell;
    d.boxbits = p_boxbits;
    d.oprefix = p_oprefix;
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
    TRY(dalloc(h, &d.hp_dirty, N));
    TRY(dalloc(h, &d.ovf, 1));
    {
        std::vector<int32_t> init(std::max(d.O, 1), 0);
        for (int i = 0; i < d.O; i++) init[i] = okind[i] == ZS_THING_BOX ? 10 : 200;  // Box / Wall MAX_LIFE
        int32_t* p_init;
        TRY(dupload(h, &p_init, init));
        d.hp_init = p_init;
        d.hp_chunk = std::max(1, (d.O + 31) / 32);
        d.hp_chunk_m = (uint32_t)(((1u << 20) + d.hp_chunk - 1) / d.hp_chunk);
        d.hp_chunk_m32 = (uint32_t)(((1ull << 32) + d.hp_chunk - 1) / d.hp_chunk);
        std::vector<uint32_t> full(std::max(d.OW, 1), 0u);
        for (int w = 0; w < d.OW; w++) full[w] = d.O - 32 * w >= 32 ? 0xffffffffu : ((1u << (d.O - 32 * w)) - 1u);
        uint32_t* p_full;
        TRY(dupload(h, &p_full, full));
        d.opres_full = p_full;
    }
    TRY(dalloc(h, &d.obst_present, (size_t)d.OW * N));
    TRY(dalloc(h, &d.obst_nonpos, (size_t)d.OW * N));
    TRY(dalloc(h, &d.dead, (size_t)d.DW * N));
    TRY(dalloc(h, &d.dead_dirty, N));
    {
        std::vector<uint32_t> zero(std::max(d.DW, 1), 0u);
        uint32_t* p_zero;
        TRY(dupload(h, &p_zero, zero));
        d.dead_zero = p_zero;
        d.dead_chunk = std::max(1, (d.DW + 31) / 32);
        d.dead_chunk_m = (uint32_t)(((1u << 20) + d.dead_chunk - 1) / d.dead_chunk);
        d.dead_chunk_m32 = (uint32_t)(((1ull << 32) + d.dead_chunk - 1) / d.dead_chunk);
        // exact for every cell when cells * (w_m * W - 2^20) < 2^20 (w_m * W - 2^20 < W)
        d.w_m = (long)d.W * d.H * d.W < (1L << 20) ? (uint32_t)(((1u << 20) + d.W - 1) / d.W) : 0u;
    }
    TRY(dalloc(h, &d.ring, (size_t)ZS_RING_WORDS * N));
    TRY(dalloc(h, &d.rngst, N));
    TRY(dalloc(h, &d.seeds, N));
    TRY(dalloc(h, &d.cand, (size_t)d.ncand * N));
    h->state_words = ZS_STATE_HEADER + ZS_STATE_ENTITY_WORDS * d.E + d.E + 2 * d.O + 2 * d.A + d.DW;
    TRY(dalloc(h, &h->d_state, (size_t)h->state_words));
    TRY(dalloc(h, &h->d_seedbuf, N));
    TRY(dalloc(h, &h->d_err, 1));
    TRY(dalloc(h, &h->d_rlist[0], N));
    TRY(dalloc(h, &h->d_rlist[1], N));
    TRY(dalloc(h, &h->d_rcount, 2));
    TRY(dalloc(h, &d.resp_list, N));
    if (d.flags & ZS_FLAG_DEATH_LOG) {
        TRY(dalloc(h, &d.dlog, (size_t)N * E * 5));
        TRY(dalloc(h, &d.dlog_n, N));
        TRY(dalloc(h, &d.alog, (size_t)N * E * 2));
        TRY(dalloc(h, &d.alog_n, N));
    }
    TRY(dalloc(h, &d.resp_count, 1));
    {
        // observation images: k_obs (four envs per workgroup when their images fit 64 KiB, else one;
        // window map and staged HP while one image fits 32 KiB) and, when the step launch writes the
        // observations itself (fobs), one env's image inside the tick / reset LDS (HP staged when the
        // image still fits the MT twist buffer it aliases).  zs_launch.obs_win forces the per-cell
        // entity scan (parity tests of that path).
        const bool world = d.obs_scope == ZS_OBS_WORLD;
        const int nobs = obs_count(d.obs_scope, d.reward_mode, d.A);
        const int plane = world ? d.W * d.H : d.obs_w * d.obs_w;
        const bool win = h->ov.obs_win >= 0;
        ObsLayout L = obs_layout(nobs, plane, d.E, d.DW, d.OW, d.O, win, true);
        if (L.bytes > 32 * 1024) L = obs_layout(nobs, plane, d.E, d.DW, d.OW, d.O, win, false);
        if (L.bytes > 32 * 1024) L = obs_layout(nobs, plane, d.E, d.DW, d.OW, d.O, false, false);
        if (L.bytes > 64 * 1024) {
            free_all(h);
            delete h;
            return fail(ZS_EINVAL, "map too large for the observation kernel's LDS image");
        }
        // static tables (4 x DW words) beside the images: per k_obs workgroup, and inside the step
        // launch's image region; zs_launch.obs_stat forces the per-cell static words (parity tests)
        d.obs_stat = (rank_order && d.DW <= 1024 && h->ov.obs_stat >= 0) ? 4 * d.DW : 0;
        h->obs_l = L;
        h->obs_wpg = d.obs_stat * 4 + 4 * L.bytes <= 64 * 1024 ? 4 : 1;
        // k_obs_pipe: surroundings of width 21, 1/2/4 observations, static tables, staged HP, window
        // map, every entity on its own lane, prefetch arrays large enough (zs_launch.obs_pipe disables)
        if (!world && d.obs_w == 21 && (nobs == 1 || nobs == 2 || nobs == 4) && d.obs_stat && L.hp_cap && L.win &&
            d.O > 0 && d.E <= 64 && d.DW <= 64 * OBS_PF_D && d.O <= 64 * OBS_PF_H && d.OW <= 64 &&
            d.obs_stat * 4 + 4 * L.bytes <= 64 * 1024 && h->ov.obs_pipe >= 0) {
            h->obs_pipe = nobs;
            // two workgroups (8 waves) per CU: measured at 65536 envs, 0.350 ms per launch against 0.375
            // at 8 and 0.38 at 3-4 (a smaller set of env blocks in flight at once); one contiguous env
            // range per wave instead of the strided walk measured slower (0.383)
            h->obs_pipe_wgs = std::max(1, std::min(2, 160 * 1024 / (d.obs_stat * 4 + 4 * L.bytes)));
            if (h->ov.obs_wgs > 0) h->obs_pipe_wgs = std::min(32, (int)h->ov.obs_wgs);
        }
        // The LDS-staged 16-B store kernels (k_obs_patch, k_obs_ring; zs_obs.hpp) for k_obs_pipe's shape,
        // channels encoding.  They pay when every wave walks several envs (at 8192 envs, one env per wave,
        // k_obs_pipe's per-cell stores measured 33 vs 36 us): int64 blocks from 48 envs per CU (C3 on one
        // MI355X, k_obs_ring against k_obs_pipe: 12 288 envs 129.5 against 117.1 M env-steps/s, 16 384 123.7 /
        // 121.4, 24 576 140.1 / 134.8, 32 768 153.6 / 147.1; 8 192 138.9 against 143.9, 10 240 (fused) 150.9 /
        // 154.9; profiles/r05c_mid_sizes.log), narrower blocks at any count.  zs_launch.obs_lds = -1 keeps
        // k_obs_pipe, 1 takes them at any count.
        bool staged = false;
        if (h->obs_pipe && d.obs_enc == ZS_ENC_CHANNELS && h->ov.obs_lds >= 0) {
            const int ts = d.obs_dtype == ZS_DTYPE_I64 ? 8 : d.obs_dtype == ZS_DTYPE_I32 ? 4 : 2;
            staged = ts < 8 || (long)d.N >= 48L * 256 || h->ov.obs_lds > 0;
        }
        // k_obs_patch: k_obs_pipe's walk with the padded-table encoder and the staged flush (maps up to
        // 4095 x 4095, rows of the padded table in the workgroup's LDS).  zs_launch.obs_patch = -1 disables.
        if (staged && d.OW <= 64 && (long)(d.W + 20) * 21 < 65536 && d.H < 4096) {
            const int ts = d.obs_dtype == ZS_DTYPE_I64 ? 8 : d.obs_dtype == ZS_DTYPE_I32 ? 4 : 2;
            const size_t pb = (size_t)patch_static_bytes(d.opad_n, d.O) +
                              PATCH_WPG * (size_t)patch_wave_bytes(d.DW, d.O, obs_stage_slot_bytes(ts));
            const int pz = h->ov.obs_patch;
            const int nobs = obs_count(d.obs_scope, d.reward_mode, d.A);
            if (pb <= 160 * 1024 && pz >= 0 &&
                obs_attr(d.obs_dtype, OBSK_PATCH, nobs, 0, (int)pb) == hipSuccess) {
                h->obs_patch = 1;
                h->obs_patch_bytes = pb;
                h->obs_patch_wgs = std::max(1, (int)(160 * 1024 / pb));
                if (h->ov.obs_wgs > 0) h->obs_patch_wgs = std::min(32, (int)h->ov.obs_wgs);
            }
        }
        // k_obs_ring (zs_obs.hpp): the staged flush with dedicated writer waves.  Measured on one MI355X
        // (2 runs each): C3 (int64) observations 292 / 280 -> 285 / 273 us against its predecessor without
        // writer waves; C5 (int16) even.  Default for int64 blocks; zs_launch.obs_ring forces either.
        if (staged) {
            const int ts = d.obs_dtype == ZS_DTYPE_I64 ? 8 : d.obs_dtype == ZS_DTYPE_I32 ? 4 : 2;
            // the ring's encoders are k_obs_patch's when its tables fit (zs_launch.obs_ring_patch forces either)
            const bool patched = h->obs_patch && h->ov.obs_ring_patch >= 0;
            const size_t rb = patched ? (size_t)ring_lds_bytes(patch_static_bytes(d.opad_n, d.O), patch_enc_bytes(d.DW, d.O), ts, nobs)
                                      : (size_t)ring_lds_bytes(16 * d.DW, L.bytes, ts, nobs);
            const int rg = h->ov.obs_ring;
            // default for int64 blocks, and for int16 ones with the padded-table encoders (C5 on one MI355X,
            // 2 runs each: 215.2 / 216.5 us against k_obs_patch's 222.7 / 223.0)
            if (rb <= 160 * 1024 && (rg ? rg > 0 : ts == 8 || (patched && ts == 2))) {
                if (obs_attr(d.obs_dtype, OBSK_RING, nobs, patched ? 1 : 0, (int)rb) == hipSuccess) {
                    h->obs_ring = patched ? 2 : 1;
                    h->obs_ring_bytes = rb;
                }
            }
        }
        // k_obs_gather when the store-stream kernel does not apply (e.g. city128's 3689 obstacles):
        // window-only static words and HP instead of per-env staging.  zs_launch.obs_gather disables.
        if (!h->obs_pipe && !world && d.obs_w == 21 && (nobs == 1 || nobs == 2 || nobs == 4) &&
            h->ov.obs_gather >= 0) {
            ObsLayout G = obs_layout(nobs, plane, d.E, d.DW, d.OW, d.O, true, false);
            if (4 * G.bytes <= 64 * 1024) {
                h->obs_gather = nobs;
                h->obs_gl = G;
                // static words from the LDS tables (rank order, as obs_stat) instead of a global load
                // round per window cell
                const size_t gb = 4 * (size_t)G.bytes;
                h->obs_gather_stat = d.obs_stat && gb + 16 * (size_t)d.DW <= 64 * 1024 && h->ov.obs_gather_stat >= 0;
            }
        }
        // k_obs_pbring: k_obs_gather's window-only fetches as the encoders of a k_obs_ring-style ring, the
        // things written over the windows (C4 on one MI355X: observations 180-184 us with k_obs_gather, 151 us
        // with k_obs_pbring), when the dead-body and present rows fit the encoders' load rounds and two unit
        // slots fit beside the static tables and the encoder regions.  zs_launch.obs_ring = -1 keeps k_obs_gather.
        if (h->obs_gather && d.obs_stat && d.obs_enc == ZS_ENC_CHANNELS && d.E <= 64 && d.DW <= 64 * BRING_D &&
            d.OW <= 64 * BRING_O && h->ov.obs_ring >= 0) {
            const int ts = d.obs_dtype == ZS_DTYPE_I64 ? 8 : d.obs_dtype == ZS_DTYPE_I32 ? 4 : 2;
            const int usp = pbring_slots(d.DW, d.OW, ts, nobs, 160 * 1024);
            const size_t pbb = (size_t)pbring_fixed_bytes(d.DW, d.OW) + (size_t)usp * bring_unit_bytes(ts, nobs);
            if (usp >= 2 && obs_attr(d.obs_dtype, OBSK_BRING, nobs, 1, (int)pbb) == hipSuccess) {
                h->obs_bring = usp;
                h->obs_bring_bytes = pbb;
            }
        }
        // with the store-stream kernel available the observations are its job (measured faster than
        // writing them from the tick workgroups at both 8192 and 65536 envs); zs_launch.fobs forces them
        // into the step launch
        d.obsl = L;
        d.fobs = L.bytes + 4 * d.obs_stat <= 16 * 1024 && h->ov.fobs >= 0;
        if (h->obs_pipe && h->ov.fobs <= 0) d.fobs = 0;
        if (d.defer_respawn) d.fobs = 0;  // the observations must see k_respawn's zombies
    }
    // Fused step launch (reset work + tick in one) when the whole launch is resident at once: then
    // the step is one latency-bound round and the reset work hides under the ticks (measured: 8192
    // envs, 1 round, fused 0.097 ms vs 0.13 ms).  With many rounds per CU (65536 envs) the reset
    // image and the reset role's registers cost every tick workgroup occupancy, so the reset work
    // runs as its own short launch (0.54 ms vs 0.59 ms).  zs_launch.fused forces either.
    {
        const int obs_b = d.fobs ? d.obsl.bytes + 4 * d.obs_stat : 0;
        TRY(choose_layout(h, cfg->lanes_per_env, true, obs_b));
        // 8 lanes per env when 16 would take the fused launch past one resident round and 8 take fewer rounds
        // (C3 on one MI355X: 16 384 envs, G = 16 two rounds 133.6 M env-steps/s, G = 8 one round 148.8 M;
        // 24 576 envs fused, G = 16 140.3 M, G = 8 143.5 M; 8 192 envs stay at G = 16, one round either way;
        // profiles/r05c_mid_sizes.log)
        if (cfg->lanes_per_env <= 0 && h->G == 16 && d.E <= 16 && h->resident < h->want) {
            const int r16 = (h->want + h->resident - 1) / h->resident;
            TRY(choose_layout(h, 8, true, obs_b));
            if ((h->want + h->resident - 1) / h->resident >= r16) TRY(choose_layout(h, 16, true, obs_b));
        }
        // up to two resident rounds the fused launch still wins: the side-stream reset work outlasts the tick
        // (C3 16 384 envs: k_tick 38 us, k_reset 43 us) and the fused launch hides it under the ticks (C3 on one
        // MI355X, fused against side stream: 12 288 envs 137.2 / 129.5 M, 16 384 133.1 / 123.7, 32 768 155.3 /
        // 153.6, 49 152 165.1 / 165.5, 65 536 172.5 / 182.0; C5 16 384 153.7 / 148.3, 32 768 186.6 / 199.3;
        // profiles/r05c_mid_sizes.log)
        h->fused = h->ov.fused ? h->ov.fused > 0 : 2 * h->resident >= h->want;
        // the fused launch loads its window's first 4G words with its first load round (zs_tick.hpp EARLY): a
        // window that size costs no round trip, and the lanes' draws then reload it less often
        if (h->fused && h->ov.rw_need <= 0) d.rw_step = std::min(d.rw_cap, std::max(d.rw_step, 4 * h->G));
        if (!h->fused) {
            TRY(choose_layout(h, cfg->lanes_per_env, false, obs_b));
            // k_tick's register budget: 5 waves per SIMD (96 VGPRs, 20 B of scratch per lane) unless 6 (80
            // VGPRs, 52 B of scratch on the leader's paths) saves a round of resident workgroups.  Measured
            // on one MI355X: C3 tick 95.6 -> 91.9 us and C4 185 -> 179 us at 5; C5 (16 384 workgroups:
            // 2.7 rounds at 6 waves, 3.2 at 5) 167 -> 178 us.  zs_launch.tick_waves forces either.
            const int wgs = (d.N + 64 / h->G - 1) / (64 / h->G);
            const int lres = std::max(1, 160 * 1024 / (int)h->lds);
            auto rounds = [&](int w) {
                const int r = std::min(lres, 4 * w);
                return (wgs + 256 * r - 1) / (256 * r);
            };
            h->tick_waves = rounds(5) <= rounds(6) ? 5 : 6;
            if (h->ov.tick_waves > 0) h->tick_waves = h->ov.tick_waves == 5 ? 5 : 6;
            h->resident = std::min(h->resident, 4 * h->tick_waves);
        }
        // the reset launch stages the static spawn lists whenever they fit (no serial global loads in
        // its candidate filters); a fused launch shares the tick's choice
        d.rlists_cap = d.lists_cap;
        if (!h->fused && d.nps + d.nzs <= 4096 &&
            reset_lds_bytes(d.E, d.DW, d.ncand, d.nps + d.nzs, obs_b) <= 64 * 1024 && h->ov.reset_lists >= 0)
            d.rlists_cap = d.nps + d.nzs;
        h->reset_lds = (size_t)reset_lds_bytes(d.E, d.DW, d.ncand, d.rlists_cap, obs_b);
    }
    if (h->reset_lds > 160 * 1024) {
        free_all(h);
        delete h;
        return fail(ZS_EINVAL, "map too large for the reset kernel's LDS image");
    }
    // side-stream reset work (unfused steps; zs_launch.reset_stream keeps it on the caller's stream)
    if (!h->fused && h->ov.reset_stream >= 0) {
        h->reset_side = hipStreamCreateWithFlags(&h->s_reset, hipStreamNonBlocking) == hipSuccess &&
                        hipEventCreateWithFlags(&h->ev_rfork, hipEventDisableTiming) == hipSuccess &&
                        hipEventCreateWithFlags(&h->ev_rjoin, hipEventDisableTiming) == hipSuccess;
    }
    if (h->reset_lds > 64 * 1024 && reset_lds_attr((int)h->reset_lds) != hipSuccess) {
        free_all(h);
        delete h;
        return fail(ZS_EHIP, "cannot raise k_reset's dynamic LDS limit");
    }
    if (getenv("ZS_VERBOSE"))
        fprintf(stderr, "zs_create: N=%d E=%d G=%d step_lds=%zu resident=%d reset_lds=%zu rw_cap=%d cand_cap=%d "
                        "lists_cap=%d fused=%d fobs=%d obs_img=%d k_obs_img=%d x%d pipe=%d gather=%d pipe_wgs=%d reset_side=%d defer_respawn=%d\n",
                d.N, d.E, h->G, h->lds, h->resident, h->reset_lds, d.rw_cap, d.cand_cap, d.lists_cap, h->fused,
                d.fobs, d.obsl.bytes, h->obs_l.bytes, h->obs_wpg, h->obs_pipe, h->obs_gather, h->obs_pipe_wgs,
                h->reset_side, d.defer_respawn);
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
    // every env starts "pending reset": the first zs_step (or zs_reset) builds its world
    hipLaunchKernelGGL(k_init_pending, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, 0, d, h->d_rlist[0],
                       h->d_rcount);
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

static int launch_obs(zs_handle* h, void* obs, const uint8_t* mask, hipStream_t s, int env0 = 0, int env1 = -1) {
    const Dev& d = h->d;
    if (!obs) return ZS_OK;
    int i0 = -1, i1 = -1;
    if (h->prof) HIPCHK(hipEventRecord(prof_event(h, &i0), s));
    if (env1 < 0) env1 = d.N;
    ObsLaunch o;
    memset(&o, 0, sizeof(o));
    o.obs = obs;
    o.mask = mask;
    o.env0 = env0;
    o.env1 = env1;
    o.nobs = h->obs_pipe;
    o.L = h->obs_l;
    if (!mask && h->obs_ring) {  // encoder / writer waves, one workgroup per CU
        const int ts = d.obs_dtype == ZS_DTYPE_I64 ? 8 : d.obs_dtype == ZS_DTYPE_I32 ? 4 : 2;
        const int pair = ring_pair(ts, h->obs_pipe);
        o.kind = OBSK_RING;
        o.patched = h->obs_ring == 2;
        o.grid = (unsigned)std::min((env1 - env0 + pair - 1) / pair, 256);
        o.block = 64 * (RING_ENC + RING_WRT);
        o.lds = h->obs_ring_bytes;
    } else if (!mask && h->obs_patch) {  // every env of [env0, env1): the padded-table encoder's store stream
        o.kind = OBSK_PATCH;
        o.grid = (unsigned)std::min((env1 - env0 + PATCH_WPG - 1) / PATCH_WPG, 256 * h->obs_patch_wgs);
        o.block = 64 * PATCH_WPG;
        o.lds = h->obs_patch_bytes;
    } else if (!mask && h->obs_pipe) {  // every env of [env0, env1), registered shape: the prefetching store stream
        o.kind = OBSK_PIPE;
        o.grid = (unsigned)std::min((env1 - env0 + 3) / 4, 256 * h->obs_pipe_wgs);
        o.block = 256;
        o.lds = (size_t)d.obs_stat * 4 + 4 * (size_t)h->obs_l.bytes;
    } else if (!mask && h->obs_bring) {  // every env of [env0, env1): window-only encoders, writer waves
        const int ts = d.obs_dtype == ZS_DTYPE_I64 ? 8 : d.obs_dtype == ZS_DTYPE_I32 ? 4 : 2;
        const int pair = ring_pair(ts, h->obs_gather);
        o.kind = OBSK_BRING;
        o.nobs = h->obs_gather;
        o.grid = (unsigned)std::min((env1 - env0 + pair - 1) / pair, 256);
        o.block = 64 * (BRING_ENC + BRING_WRT);
        o.lds = h->obs_bring_bytes;
        o.L = h->obs_gl;
        o.us = h->obs_bring;
    } else if (h->obs_gather) {  // one env per wave, four per workgroup, window-only fetches
        o.kind = OBSK_GATHER;
        o.nobs = h->obs_gather;
        o.grid = (unsigned)((d.N + 3) / 4);
        o.block = 256;
        o.lds = 4 * (size_t)h->obs_gl.bytes + (h->obs_gather_stat ? 16 * (size_t)d.DW : 0);
        o.L = h->obs_gl;
        o.stat = h->obs_gather_stat;
    } else {
        o.kind = OBSK_OBS;
        o.grid = (unsigned)((d.N + h->obs_wpg - 1) / h->obs_wpg);
        o.block = 64 * h->obs_wpg;
        o.lds = (size_t)d.obs_stat * 4 + (size_t)h->obs_wpg * h->obs_l.bytes;
        o.stat = d.obs_stat;
    }
    HIPCHK(obs_launch(d.obs_dtype, o, s, d));
    if (h->prof) {
        HIPCHK(hipEventRecord(prof_event(h, &i1), s));
        h->ev_obs.push_back({i0, i1});
    }
    return ZS_OK;
}

static int launch_tick(zs_handle* h, const int32_t* actions, double* rew, uint8_t* done, uint8_t* trunc,
                       uint8_t* listed, uint8_t* reset_out, int* rlist, int* rcount, void* obs, hipStream_t s,
                       int env0 = 0, int env1 = -1) {
    const Dev& d = h->d;
    const int ne = 64 / h->G;
    if (env1 < 0) env1 = d.N;
    unsigned grid = (unsigned)((env1 - env0 + ne - 1) / ne);
    int i0 = -1, i1 = -1;
    const int p = h->rpar;
    // fused: the first n_reset workgroups rebuild the envs of the pending list (ended at the previous
    // call) while the others tick every other env; the two sets of envs are disjoint
    const int n_reset = std::min(d.N, reset_wgs(h));
    if (h->prof) HIPCHK(hipEventRecord(prof_event(h, &i0), s));
    TickArgs a;
    a.actions = actions;
    a.rew = rew;
    a.done = done;
    a.trunc = trunc;
    a.listed = listed;
    a.reset_out = reset_out;
    a.rlist = rlist;
    a.rcount = rcount;
    a.obs = obs;
    a.env0 = env0;
    a.env1 = env1;
    a.n_reset = h->fused ? n_reset : 0;
    a.cur_list = (const int*)h->d_rlist[p];
    a.cur_count = (const int*)(h->d_rcount + p);
    a.err = h->d_err;
    hipError_t le;
    switch (h->G) {
    case 1: le = launch_tick_g1(h->fused, h->tick_waves, grid, h->lds, s, d, a); break;
    case 2: le = launch_tick_g2(h->fused, h->tick_waves, grid, h->lds, s, d, a); break;
    case 4: le = launch_tick_g4(h->fused, h->tick_waves, grid, h->lds, s, d, a); break;
    case 8: le = launch_tick_g8(h->fused, h->tick_waves, grid, h->lds, s, d, a); break;
    case 16: le = launch_tick_g16(h->fused, h->tick_waves, grid, h->lds, s, d, a); break;
    case 32: le = launch_tick_g32(h->fused, h->tick_waves, grid, h->lds, s, d, a); break;
    default: le = launch_tick_g64(h->fused, h->tick_waves, grid, h->lds, s, d, a); break;
    }
    HIPCHK(le);
    if (h->prof) {
        HIPCHK(hipEventRecord(prof_event(h, &i1), s));
        h->ev_tick.push_back({i0, i1});
    }
    return ZS_OK;
}

static int launch_reset(zs_handle* h, int list_mode, const uint8_t* mask, void* obs, hipStream_t s) {
    const Dev& d = h->d;
    // enough one-wave workgroups that a step's resets (~850 at 65536 envs, bridge64) run in one round
    const int rgrid = h->ov.reset_grid > 0 ? h->ov.reset_grid : 2048;
    unsigned grid = (unsigned)std::min(d.N, list_mode ? rgrid : 4096);
    int p = h->rpar;
    int i0 = -1, i1 = -1;
    if (h->prof) HIPCHK(hipEventRecord(prof_event(h, &i0), s));
    HIPCHK(launch_reset_k(grid, h->reset_lds, s, d, list_mode, h->d_rlist[p], h->d_rcount + p, mask, h->d_err, obs));
    if (h->prof) {
        HIPCHK(hipEventRecord(prof_event(h, &i1), s));
        h->ev_reset.push_back({i0, i1});
    }
    return ZS_OK;
}

// the respawns the tick just deferred (k_respawn drains d.resp_list; count zeroed before the tick)
static int launch_respawn(zs_handle* h, hipStream_t s) {
    const Dev& d = h->d;
    // enough one-wave workgroups for a step's respawns in one pass (C4: 2048 -> 8192 took the launch
    // from 88 to 70 us; workgroups past the list's end exit at once)
    const int grid = h->ov.respawn_grid > 0 ? h->ov.respawn_grid : 8192;
    int i0 = -1, i1 = -1;
    if (h->prof) HIPCHK(hipEventRecord(prof_event(h, &i0), s));
    HIPCHK(launch_respawn_k((unsigned)std::min(d.N, grid), h->reset_lds, s, d));
    if (h->prof) {
        HIPCHK(hipEventRecord(prof_event(h, &i1), s));
        h->ev_respawn.push_back({i0, i1});
    }
    return ZS_OK;
}

// zs_reset's launches, queued on s (the caller synchronises and reads h->d_err)
static int queue_reset(zs_handle* h, const uint8_t* env_mask_dev, void* obs_dev, hipStream_t s) {
    HIPCHK(hipMemsetAsync(h->d_err, 0, sizeof(int), s));
    int rc = launch_reset(h, 0, env_mask_dev, nullptr, s);
    if (rc) return rc;
    // the pending-reset list must hold exactly the envs still pending: drop the ones just rebuilt
    {
        int p = h->rpar, q = 1 - p;
        if (!env_mask_dev) {
            HIPCHK(hipMemsetAsync(h->d_rcount + p, 0, sizeof(int), s));
        } else {
            HIPCHK(hipMemsetAsync(h->d_rcount + q, 0, sizeof(int), s));
            HIPCHK(launch_list_filter((unsigned)std::min(64, (h->d.N + 255) / 256), s, (const int*)h->d_rlist[p],
                                      (const int*)(h->d_rcount + p), h->d_rlist[q], h->d_rcount + q, env_mask_dev,
                                      h->d.N));
            // the list the next step appends to (list[p] now) starts empty (zs_step's counter protocol)
            HIPCHK(hipMemsetAsync(h->d_rcount + p, 0, sizeof(int), s));
            h->rpar = q;
        }
    }
    return launch_obs(h, obs_dev, env_mask_dev, s);
}

extern "C" int zs_reset(zs_handle* h, const uint8_t* env_mask_dev, void* obs_dev, void* stream) {
    if (!h) return fail(ZS_EINVAL, "null handle");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    int rc = queue_reset(h, env_mask_dev, obs_dev, s);
    if (rc) return rc;
    int err = 0;
    HIPCHK(hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemsetAsync(h->d_err, 0, sizeof(int), s));  // every reader leaves the error word clear
    HIPCHK(hipStreamSynchronize(s));
    if (err == ZS_ENOSPACE) return fail(ZS_ENOSPACE, "Not enough space to spawn players/agents");
    if (err) return fail(err, "reset failed");
    return ZS_OK;
}

// Observation only (the reference's env.get_observation(), gym_env.py:93-94): re-encode the
// current state of the masked envs, e.g. after a zs_set_state poke.
extern "C" int zs_observe(zs_handle* h, const uint8_t* env_mask_dev, void* obs_dev, void* stream) {
    if (!h || !obs_dev) return fail(ZS_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    return launch_obs(h, obs_dev, env_mask_dev, s);
}

extern "C" int zs_step(zs_handle* h, const int32_t* actions_dev, void* obs_dev, double* rewards_dev, uint8_t* done_dev,
                       uint8_t* trunc_dev, uint8_t* listed_dev, uint8_t* reset_dev, void* stream) {
    if (!h || !actions_dev || !rewards_dev || !done_dev || !trunc_dev) return fail(ZS_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    // 1) rebuild the envs that ended at the previous call (list[p]); fused into the tick launch
    //    when the LDS images allow, else a k_reset launch first
    int q = 1 - h->rpar, rc = ZS_OK;
    bool side = false;
    if (!h->fused) {
        side = h->reset_side != 0;
        hipStream_t rs = s;
        if (side) {  // fork: the reset work sees everything the caller queued before this call
            HIPCHK(hipEventRecord(h->ev_rfork, s));
            HIPCHK(hipStreamWaitEvent(h->s_reset, h->ev_rfork, 0));
            rs = h->s_reset;
        }
        // zs_step_graph's policy: with the reset work beside the tick, its own launch on the caller's
        // stream right after the fork and ahead of the reset launch (captured in that order, the graph
        // starts the policy first: C3 173 M env-steps/s, against 167 with the reset launch captured first
        // and 169 with the policy inside the step launch); otherwise inside the step launch (no launch,
        // no gap: 8 192 envs 110 -> 117 M env-steps/s)
        if (h->graph_pol && side) {
            const int n = h->d.N * h->d.A;
            hipLaunchKernelGGL(k_gen_actions_ctr, dim3((n + 255) / 256), dim3(256), 0, s, h->d,
                               (const uint64_t*)h->d_gstep, h->graph_pol, (int32_t*)actions_dev);
            HIPCHK(hipGetLastError());
        }
        rc = launch_reset(h, 1, nullptr, h->d.fobs ? obs_dev : nullptr, rs);
        if (rc) return rc;
        if (side) HIPCHK(hipEventRecord(h->ev_rjoin, h->s_reset));
    }
    struct PolScope {
        Dev& d;
        PolScope(Dev& dd, int n, const uint64_t* st) : d(dd) {
            d.pol_n = n;
            d.pol_step = st;
        }
        ~PolScope() { d.pol_n = 0, d.pol_step = nullptr; }
    } pol(h->d, side ? 0 : h->graph_pol, side ? nullptr : h->d_gstep);
    // 2) tick every other env; envs that end now are queued on list[q] for the next call.
    // Work-list counters: between calls the list the next step appends to (list[1 - rpar]) and the
    // deferred-respawn list are empty.  This step appends to list[q] and resp_list, drains list[p] and
    // resp_list, and its last launch (the observation kernel, else k_tail) empties list[p] and resp_list
    // again (Dev::tail_*), so no launch ahead of the tick is needed.  (Not by captured 4-byte
    // hipMemsetAsync nodes: in this engine's round-2 city128 graph such nodes left byte patterns in the
    // counters, profiles/r02_graph_memset_city128.log; tools/probe/graphprobe.hip replays that node
    // sequence standalone without a fault, profiles/r03_graphprobe_fork.log.)  Every list index is
    // bounds-checked in the kernels.
    const int p = h->rpar;
    rc = launch_tick(h, actions_dev, rewards_dev, done_dev, trunc_dev, listed_dev, reset_dev, h->d_rlist[q],
                     h->d_rcount + q, obs_dev, s);
    if (rc) return rc;
    h->rpar = q;
    // a launch failing after the tick was queued: the step's tail (the counter protocol above) is done
    // here instead, so the next step does not append after stale counts (not while capturing: a failed
    // capture is discarded, and nothing of it ran)
    auto tail_on_error = [&](int code) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
            (void)hipMemsetAsync(h->d_rcount + p, 0, sizeof(int), s);
            if (h->d.defer_respawn) (void)hipMemsetAsync(h->d.resp_count, 0, sizeof(int), s);
        }
        return code;
    };
    if (h->d.defer_respawn) {
        rc = launch_respawn(h, s);
        if (rc) return tail_on_error(rc);
    }
    // join the reset work, then 3) observations of every env (already written by the step launch
    // when fobs), carrying the step's tail
    if (side && hipStreamWaitEvent(s, h->ev_rjoin, 0) != hipSuccess) return tail_on_error(fail(ZS_EHIP, "hipStreamWaitEvent"));
    struct TailScope {
        Dev& d;
        TailScope(Dev& dd, int* c0, int* c1, uint64_t* st) : d(dd) {
            d.tail_cnt0 = c0;
            d.tail_cnt1 = c1;
            d.tail_step = st;
        }
        ~TailScope() { d.tail_cnt0 = d.tail_cnt1 = nullptr, d.tail_step = nullptr; }
    } tail(h->d, h->d_rcount + p, h->d.defer_respawn ? h->d.resp_count : nullptr, h->graph_pol ? h->d_gstep : nullptr);
    if (h->d.fobs || !obs_dev) {
        hipLaunchKernelGGL(k_tail, dim3(1), dim3(64), 0, s, h->d);
        const hipError_t le = hipGetLastError();
        return le == hipSuccess ? ZS_OK : tail_on_error(fail(ZS_EHIP, std::string("k_tail: ") + hipGetErrorString(le)));
    }
    rc = launch_obs(h, obs_dev, nullptr, s);
    return rc ? tail_on_error(rc) : ZS_OK;
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

// One step of the on-device policy loop (zs_gen_actions for the next step number, then zs_step) as a
// replayed hipGraph: the launches of a step are captured once per pending-list parity and then
// cost one graph launch per step instead of one dispatch each.  step0 is the step number of the
// first call after (re)capture; later calls continue from the device counter.
extern "C" int zs_step_graph(zs_handle* h, uint64_t step0, int32_t n_discrete, int32_t* actions_dev, void* obs_dev,
                             double* rewards_dev, uint8_t* done_dev, uint8_t* trunc_dev, uint8_t* listed_dev,
                             uint8_t* reset_dev, void* stream) {
    return zs_step_graph_n(h, step0, n_discrete, 1, actions_dev, obs_dev, rewards_dev, done_dev, trunc_dev, listed_dev,
                           reset_dev, stream);
}

extern "C" int zs_step_graph_n(zs_handle* h, uint64_t step0, int32_t n_discrete, int32_t n_steps, int32_t* actions_dev,
                               void* obs_dev, double* rewards_dev, uint8_t* done_dev, uint8_t* trunc_dev,
                               uint8_t* listed_dev, uint8_t* reset_dev, void* stream) {
    if (!h || !actions_dev || !rewards_dev || !done_dev || !trunc_dev) return fail(ZS_EINVAL, "null argument");
    // n_discrete = 0: the caller's actions (no policy launch; the graph replays zs_step on actions_dev)
    if (n_discrete < 0 || n_discrete > 7) return fail(ZS_EINVAL, "n_discrete must be in 0..7");
    if (n_steps < 1 || n_steps > 64) return fail(ZS_EINVAL, "n_steps must be in 1..64");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    const void* key[9] = {actions_dev, obs_dev, rewards_dev, done_dev, trunc_dev, listed_dev, reset_dev,
                          (const void*)(intptr_t)n_discrete, (const void*)(intptr_t)n_steps};
    zs_handle::GraphSet* set = nullptr;
    for (auto& gs : h->gsets) {
        bool same = gs.g[0] && gs.g[1];
        for (int k = 0; k < 9 && same; k++) same = key[k] == gs.key[k];
        if (same) set = &gs;
    }
    if (!set) {  // capture into the least recently used set
        set = &h->gsets[0];
        for (auto& gs : h->gsets)
            if (gs.used < set->used) set = &gs;
        for (hipGraphExec_t& g : set->g)
            if (g) {
                HIPCHK(hipGraphExecDestroy(g));
                g = nullptr;
            }
        if (!h->d_gstep) {
            int rc = dalloc(h, &h->d_gstep, 2);
            if (rc) return rc;
        }
        uint64_t init[2] = {step0, 0};
        HIPCHK(hipMemcpyAsync(h->d_gstep, init, sizeof(init), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        hipStream_t cs;
        HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        const int prof = h->prof;
        h->prof = 0;  // no timing events inside a graph
        const int p0 = h->rpar;
        int rc = ZS_OK;
        for (int g = 0; g < 2 && rc == ZS_OK; g++) {  // starting parity p0, then 1 - p0 (zs_step flips rpar)
            hipGraph_t graph = nullptr;
            h->rpar = (p0 + g) & 1;
            if (hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) != hipSuccess) {
                rc = fail(ZS_EHIP, "hipStreamBeginCapture failed");
                break;
            }
            // each step's policy reads the step number *d_gstep (zs_step: its own launch, or inside the
            // step launch), the step's tail advances it
            h->graph_pol = n_discrete;
            for (int k = 0; k < n_steps && rc == ZS_OK; k++)
                rc = zs_step(h, actions_dev, obs_dev, rewards_dev, done_dev, trunc_dev, listed_dev, reset_dev, cs);
            h->graph_pol = 0;
            hipError_t ce = hipStreamEndCapture(cs, &graph);
            if (rc == ZS_OK && ce != hipSuccess) rc = fail(ZS_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
            if (rc == ZS_OK) {
                hipError_t ie = hipGraphInstantiate(&set->g[(p0 + g) & 1], graph, nullptr, nullptr, 0);
                if (ie != hipSuccess) rc = fail(ZS_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
            }
            if (graph) (void)hipGraphDestroy(graph);
        }
        h->rpar = p0;  // a capture runs no work: the lists are where they were
        h->prof = prof;
        (void)hipStreamDestroy(cs);
        if (rc != ZS_OK) {
            for (hipGraphExec_t& g : set->g)
                if (g) {
                    (void)hipGraphExecDestroy(g);
                    g = nullptr;
                }
            return rc;
        }
        for (int k = 0; k < 9; k++) set->key[k] = key[k];
    }
    set->used = ++h->gclock;
    // g[p] starts by draining list p (the parity of its first step); each step flips the parity
    HIPCHK(hipGraphLaunch(set->g[h->rpar], s));
    h->rpar ^= n_steps & 1;
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
    {  // a present thing stands on a map cell (the occupancy and observation kernels index the map by it)
        const int32_t* r = buf_host + ZS_STATE_HEADER;
        for (int s = 0; s < h->d.E; s++, r += ZS_STATE_ENTITY_WORDS)
            if (r[1] && (r[2] < 0 || r[3] < 0 || r[2] >= h->d.W || r[3] >= h->d.H))
                return fail(ZS_EINVAL, "a present entity's position is outside the map");
    }
    {  // obstacle life is int32 in HBM; INT32_MIN is the observation kernels' absent mark (ZS_HP_FLOOR)
        const int32_t* hp = buf_host + ZS_STATE_HEADER + ZS_STATE_ENTITY_WORDS * h->d.E + h->d.E;
        for (int o = 0; o < h->d.O; o++)
            if (hp[o] < ZS_HP_FLOOR) return fail(ZS_EINVAL, "obstacle life below -2147483647");
    }
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMemsetAsync(h->d_err, 0, sizeof(int), s));
    HIPCHK(hipMemcpyAsync(h->d_state, buf_host, sizeof(int32_t) * h->state_words, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_set_state, dim3(1), dim3(64), 0, s, h->d, env, h->d_state, h->d_err);
    HIPCHK(hipGetLastError());
    int err = 0;
    HIPCHK(hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemsetAsync(h->d_err, 0, sizeof(int), s));
    HIPCHK(hipStreamSynchronize(s));
    if (err) return fail(ZS_EINVAL, "state record's needs_reset [5] differs from the engine's (pending resets are not settable)");
    return ZS_OK;
}

extern "C" int zs_overflow(zs_handle* h, uint32_t* flags_host, int32_t clear, void* stream) {
    if (!h || !flags_host) return fail(ZS_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    uint32_t f = 0;
    HIPCHK(hipMemcpyAsync(&f, h->d.ovf, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (clear) HIPCHK(hipMemsetAsync(h->d.ovf, 0, sizeof(uint32_t), s));
    HIPCHK(hipStreamSynchronize(s));
    *flags_host = f;
    return ZS_OK;
}

// ---------------------------------------------------------------------------
// An env's MT19937 stream in CPython's random.getstate() form: state[0..623] = the raw
// block being consumed, state[624] = index of the next word (0..624; 624 = exhausted, the
// next draw twists).  The single-env wrappers move the process-global `random` state in
// and out of the engine around every call, so the engine draws from exactly the stream the
// reference's `random` module would (one process-global RNG).
// ---------------------------------------------------------------------------
extern "C" int zs_get_rng(zs_handle* h, int32_t env, uint32_t* state_host, void* stream) {
    if (!h || !state_host) return fail(ZS_EINVAL, "null argument");
    if (env < 0 || env >= h->d.N) return fail(ZS_EINVAL, "env index out of range");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    uint32_t st = 0;
    std::vector<uint32_t> ring(ZS_RING_WORDS);
    HIPCHK(hipMemcpyAsync(&st, h->d.rngst + env, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(ring.data(), h->d.ring + (size_t)env * ZS_RING_WORDS, sizeof(uint32_t) * ZS_RING_WORDS,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    uint32_t off = st & 1023u, slot = (st >> 10) & 1u;
    std::memcpy(state_host, ring.data() + slot * ZS_MT_N, sizeof(uint32_t) * ZS_MT_N);
    state_host[ZS_MT_N] = off;
    return ZS_OK;
}

extern "C" int zs_set_rng(zs_handle* h, int32_t env, const uint32_t* state_host, void* stream) {
    if (!h || !state_host) return fail(ZS_EINVAL, "null argument");
    if (env < 0 || env >= h->d.N) return fail(ZS_EINVAL, "env index out of range");
    if (state_host[ZS_MT_N] > ZS_MT_N) return fail(ZS_EINVAL, "MT index out of range (0..624)");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    // slot 0 = the given block, slot 1 = its successor (x[k+624] = x[k+397] ^ f(x[k], x[k+1]))
    std::vector<uint32_t> ring(ZS_RING_WORDS);
    std::memcpy(ring.data(), state_host, sizeof(uint32_t) * ZS_MT_N);
    for (int k = 0; k < ZS_MT_N; k++) {
        uint32_t a = ring[k], b = ring[k + 1], c = ring[k + ZS_MT_M];
        uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
        ring[ZS_MT_N + k] = c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    uint32_t st = state_host[ZS_MT_N] | (0u << 10) | (1u << 11);
    HIPCHK(hipMemcpyAsync(h->d.ring + (size_t)env * ZS_RING_WORDS, ring.data(), sizeof(uint32_t) * ZS_RING_WORDS,
                          hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(h->d.rngst + env, &st, sizeof(uint32_t), hipMemcpyHostToDevice, s));
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
    h->ev_reset.clear();
    h->ev_respawn.clear();
    h->ev_next = 0;
    return ZS_OK;
}

extern "C" int zs_profile_read(zs_handle* h, double* out) {
    if (!h || !out) return fail(ZS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(h->device));
    double tot[4] = {0.0, 0.0, 0.0, 0.0};
    std::vector<std::pair<int, int>>* lists[4] = {&h->ev_tick, &h->ev_obs, &h->ev_reset, &h->ev_respawn};
    for (int k = 0; k < 4; k++)
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
    out[4] = tot[2];
    out[5] = (double)h->ev_reset.size();
    out[6] = tot[3];
    out[7] = (double)h->ev_respawn.size();
    h->ev_tick.clear();
    h->ev_obs.clear();
    h->ev_reset.clear();
    h->ev_respawn.clear();
    h->ev_next = 0;
    return ZS_OK;
}

extern "C" int zs_describe(zs_handle* h, char* buf, int32_t len) {
    if (!h || !buf || len <= 0) return fail(ZS_EINVAL, "null argument");
    const Dev& d = h->d;
    const char* obs_kernel = d.fobs ? "step launch"
                             : h->obs_pipe ? (h->obs_ring ? "k_obs_ring" : h->obs_patch ? "k_obs_patch" : "k_obs_pipe")
                             : h->obs_bring ? "k_obs_pbring" : h->obs_gather ? "k_obs_gather" : "k_obs";
    snprintf(buf, (size_t)len,
             "{\"envs\": %d, \"entities\": %d, \"lanes_per_env\": %d, \"step_kernel\": \"%s\", \"step_lds\": %zu, "
             "\"step_wgs_per_cu\": %d, \"rng_window\": %d, \"obs_kernel\": \"%s\", \"reset_side_stream\": %d, "
             "\"reset_lds\": %zu, \"respawn\": \"%s\", \"tick_waves\": %d, \"rng_step\": %d, \"par_exec\": %d}",
             d.N, d.E, h->G, h->fused ? "k_step" : "k_tick", h->lds, h->resident, d.rw_cap, obs_kernel,
             h->reset_side,
             h->reset_lds, d.defer_respawn ? "k_respawn" : "tick", h->fused ? ZS_FUSED_WAVES : h->tick_waves, d.rw_step,
             d.par_exec);
    return ZS_OK;
}

// The actions env's last step executed, in execution order (the shuffled action list of World.step,
// core.py:76,103-119): per action {slot | kind << 8, target}, kind 1 move (target: the destination,
// x | y << 16), 2 attack, 3 heal (target: an entity slot, or -1 - obstacle index).  Needs ZS_FLAG_DEATH_LOG.
extern "C" int zs_action_log(zs_handle* h, int32_t env, int32_t* out_host, int32_t cap, int32_t* n_out, void* stream) {
    if (!h || !n_out || (cap > 0 && !out_host)) return fail(ZS_EINVAL, "null argument");
    if (!h->d.alog) return fail(ZS_EINVAL, "the handle was created without ZS_FLAG_DEATH_LOG");
    if (env < 0 || env >= h->d.N) return fail(ZS_EINVAL, "env out of range");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    int32_t n = 0;
    HIPCHK(hipMemcpyAsync(&n, h->d.alog_n + env, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    // n < 0: a debug raise stopped the step; -1 - n actors before the raising one decided an action
    n = std::max(-1 - h->d.E, std::min(n, h->d.E));
    const int k = std::min(n < 0 ? -1 - n : n, std::max(0, (int)cap));
    if (k > 0) {
        HIPCHK(hipMemcpyAsync(out_host, h->d.alog + (size_t)env * h->d.E * 2, sizeof(int32_t) * 2 * k,
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    *n_out = n;
    return ZS_OK;
}

extern "C" int zs_death_log(zs_handle* h, int32_t env, int32_t* out_host, int32_t cap, int32_t* n_out, void* stream) {
    if (!h || !n_out || (cap > 0 && !out_host)) return fail(ZS_EINVAL, "null argument");
    if (!h->d.dlog) return fail(ZS_EINVAL, "the handle was created without ZS_FLAG_DEATH_LOG");
    if (env < 0 || env >= h->d.N) return fail(ZS_EINVAL, "env out of range");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    int32_t n = 0;
    HIPCHK(hipMemcpyAsync(&n, h->d.dlog_n + env, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    n = std::max(0, std::min(n, h->d.E));
    const int k = std::min(n, std::max(0, (int)cap));
    if (k > 0) {
        HIPCHK(hipMemcpyAsync(out_host, h->d.dlog + (size_t)env * h->d.E * 5, sizeof(int32_t) * 5 * k,
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    *n_out = n;
    return ZS_OK;
}

// ---------------------------------------------------------------------------
// The drop-ins' per-call path.  The reference's env.step / env.reset / env.get_observation run one env
// per call on the host (gym_env.py:99-164, gym/multiagent_env.py:111-184) and share the process-global
// `random` stream.  Here one call is: the caller's actions and `random` state written into one pinned,
// device-mapped block that the kernels read in place, the engine's launches, k_host_pack writing
// everything the host reads back (outputs, the advanced stream, the action / death logs, the state
// record, the observation) into one pinned, device-mapped record per env, and one synchronisation.
// ---------------------------------------------------------------------------
static int obs_bytes_per_env(const zs_handle* h) {
    int32_t shp[4];
    zs_obs_shape(h, shp);
    const int ts = h->d.obs_dtype == ZS_DTYPE_I64 ? 8 : h->d.obs_dtype == ZS_DTYPE_I32 ? 4 : 2;
    return shp[0] * shp[1] * shp[2] * shp[3] * ts;
}

static HostLayout host_layout(const zs_handle* h) {
    const Dev& d = h->d;
    HostLayout L;
    L.R = d.reward_mode == ZS_REWARD_SINGLE ? 1 : d.A;
    L.obs_bytes = obs_bytes_per_env(h);
    L.rew = ZS_HOST_RNG + ZS_MT_N + 2;  // even: the rewards are float64
    L.alog = L.rew + 2 * L.R;
    L.dlog = L.alog + 2 * d.E;
    L.state = L.dlog + 5 * d.E;
    L.obs = (L.state + h->state_words + 3) & ~3;  // 16-byte aligned
    L.words = (L.obs + (L.obs_bytes + 3) / 4 + 3) & ~3;
    return L;
}

static int host_init(zs_handle* h) {
    if (h->d_hrec) return ZS_OK;
    const Dev& d = h->d;
    const size_t N = d.N;
    HostLayout L = host_layout(h);
    const size_t in_words = N * d.A * 3 + N * (ZS_RING_WORDS + 1);
    int rc;
    if ((rc = dalloc(h, &h->d_hobs, N * L.obs_bytes)) || (rc = dalloc(h, &h->d_hrew, N * L.R)) ||
        (rc = dalloc(h, &h->d_hflags, N * (3 + d.A))))
        return rc;
    // coherent (uncached on the device) so the kernels see this call's input and the host the record
    // without copies; the blocks are a few KB per env
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    HIPCHK(hipHostMalloc((void**)&h->h_hin, in_words * sizeof(int32_t), fl));
    HIPCHK(hipHostMalloc((void**)&h->h_hrec, N * L.words * sizeof(int32_t), fl));
    HIPCHK(hipHostGetDevicePointer((void**)&h->d_hin, h->h_hin, 0));
    HIPCHK(hipHostGetDevicePointer((void**)&h->d_hrec, h->h_hrec, 0));
    h->hl = L;
    return ZS_OK;
}

// the `random` states of envs [0, N) (CPython getstate() form, 625 words each) into the pinned input
// block after the actions: per env its ring (the block, then its successor) and its st word
static int host_stage_rng(zs_handle* h, const uint32_t* rng_host) {
    const size_t N = h->d.N;
    uint32_t* rings = (uint32_t*)h->h_hin + N * h->d.A * 3;
    uint32_t* st = rings + N * ZS_RING_WORDS;
    for (size_t e = 0; e < N; e++) {
        const uint32_t* g = rng_host + e * (ZS_MT_N + 1);
        if (g[ZS_MT_N] > ZS_MT_N) return fail(ZS_EINVAL, "MT index out of range (0..624)");
        uint32_t* r = rings + e * ZS_RING_WORDS;
        std::memcpy(r, g, sizeof(uint32_t) * ZS_MT_N);
        for (int k = 0; k < ZS_MT_N; k++) {  // x[k+624] = x[k+397] ^ f(x[k], x[k+1])
            uint32_t a = r[k], b = r[k + 1], c = r[k + ZS_MT_M];
            uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            r[ZS_MT_N + k] = c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        st[e] = g[ZS_MT_N] | (0u << 10) | (1u << 11);
    }
    return ZS_OK;
}

enum { HOST_STEP = 0, HOST_RESET = 1, HOST_OBSERVE = 2 };

static int host_call(zs_handle* h, int op, const int32_t* actions_host, const uint32_t* rng_host, int32_t* rec_host,
                     hipStream_t s) {
    HIPCHK(hipSetDevice(h->device));
    int rc = host_init(h);
    if (rc) return rc;
    const Dev& d = h->d;
    const size_t N = d.N;
    const HostLayout& L = h->hl;
    if (op == HOST_STEP) std::memcpy(h->h_hin, actions_host, sizeof(int32_t) * N * d.A * 3);
    if (rng_host && (rc = host_stage_rng(h, rng_host))) return rc;
    if (rng_host) {
        const uint32_t* rings = (const uint32_t*)h->d_hin + N * d.A * 3;
        hipLaunchKernelGGL(k_host_unpack, dim3((unsigned)N), dim3(256), 0, s, h->d, rings, rings + N * ZS_RING_WORDS);
        HIPCHK(hipGetLastError());
    }
    uint8_t *done = h->d_hflags, *trunc = done + N, *rst = trunc + N, *listed = rst + N;
    if (op == HOST_STEP) {  // (d_err is clear: k_host_pack clears it, and zs_reset / zs_set_state before use)
        rc = zs_step(h, h->d_hin, h->d_hobs, h->d_hrew, done, trunc, listed, rst, s);
    } else if (op == HOST_RESET) {
        HIPCHK(hipMemsetAsync(h->d_hflags, 0, N * 3, s));
        HIPCHK(hipMemsetAsync(h->d_hrew, 0, N * L.R * sizeof(double), s));
        rc = queue_reset(h, nullptr, h->d_hobs, s);
    } else {
        rc = launch_obs(h, h->d_hobs, nullptr, s);
    }
    if (rc) return rc;
    hipLaunchKernelGGL(k_host_pack, dim3((unsigned)N), dim3(256), 0, s, h->d, L, (const uint8_t*)h->d_hobs,
                       (const double*)h->d_hrew, (const uint8_t*)done, (const uint8_t*)trunc,
                       op == HOST_RESET ? nullptr : (const uint8_t*)rst, h->d_err, h->d_hrec);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    std::memcpy(rec_host, h->h_hrec, N * L.words * sizeof(int32_t));
    const int err = h->h_hrec[ZS_HOST_ERR];
    if (err == ZS_ENOSPACE) return fail(ZS_ENOSPACE, "Not enough space to spawn players/agents");
    if (err) return fail(err, "reset failed");
    return ZS_OK;
}

extern "C" int zs_host_layout(zs_handle* h, int32_t out[8]) {
    if (!h || !out) return fail(ZS_EINVAL, "null argument");
    const HostLayout L = host_layout(h);
    const int32_t v[8] = {L.words, L.rew, L.alog, L.dlog, L.state, L.obs, L.obs_bytes, L.R};
    std::memcpy(out, v, sizeof(v));
    return ZS_OK;
}

extern "C" int zs_host_step(zs_handle* h, const int32_t* actions_host, const uint32_t* rng_host, int32_t* rec_host,
                            void* stream) {
    if (!h || !actions_host || !rec_host) return fail(ZS_EINVAL, "null argument");
    return host_call(h, HOST_STEP, actions_host, rng_host, rec_host, (hipStream_t)stream);
}

extern "C" int zs_host_reset(zs_handle* h, const uint32_t* rng_host, int32_t* rec_host, void* stream) {
    if (!h || !rec_host) return fail(ZS_EINVAL, "null argument");
    return host_call(h, HOST_RESET, nullptr, rng_host, rec_host, (hipStream_t)stream);
}

extern "C" int zs_host_observe(zs_handle* h, int32_t* rec_host, void* stream) {
    if (!h || !rec_host) return fail(ZS_EINVAL, "null argument");
    return host_call(h, HOST_OBSERVE, nullptr, nullptr, rec_host, (hipStream_t)stream);
}

// Diagnostics: the work-list counters as they stand after everything queued on `stream` (out[0..1]
// the two pending-reset list counts, out[2] the deferred-respawn count, out[3] the parity the next
// step drains).
extern "C" int zs_debug_lists(zs_handle* h, int32_t* out, void* stream) {
    if (!h || !out) return fail(ZS_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    int v[3] = {0, 0, 0};
    HIPCHK(hipMemcpyAsync(v, h->d_rcount, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(v + 2, h->d.resp_count, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    out[0] = v[0];
    out[1] = v[1];
    out[2] = v[2];
    out[3] = h->rpar;
    return ZS_OK;
}

// ---------------------------------------------------------------------------
// diagnostic build (-DZS_STAMPS): per-phase k_tick cycle sums since the last read
// ---------------------------------------------------------------------------
#ifdef ZS_STAMPS
// this handle's step-kernel unit (its G)
static hipError_t stamps_of(int G, unsigned long long* wg, unsigned long long* tl, int clear) {
    switch (G) {
    case 1: return stamps_g1(wg, tl, clear);
    case 2: return stamps_g2(wg, tl, clear);
    case 4: return stamps_g4(wg, tl, clear);
    case 8: return stamps_g8(wg, tl, clear);
    case 16: return stamps_g16(wg, tl, clear);
    case 32: return stamps_g32(wg, tl, clear);
    default: return stamps_g64(wg, tl, clear);
    }
}
#endif

// diagnostic build (-DZS_STAMPS): start / end s_memrealtime of the first n workgroups of the last step launch
extern "C" int zs_debug_timeline(zs_handle* h, uint64_t* out, int32_t n) {
#ifdef ZS_STAMPS
    if (!h || !out || n < 0 || n > ZS_STAMP_WGS) return fail(ZS_EINVAL, "bad argument");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> tl((size_t)ZS_STAMP_WGS * 2);
    HIPCHK(stamps_of(h->G, nullptr, tl.data(), 0));
    std::memcpy(out, tl.data(), (size_t)n * 2 * sizeof(unsigned long long));
    return ZS_OK;
#else
    (void)h; (void)out; (void)n;
    return fail(ZS_ESTATE, "not a ZS_STAMPS diagnostic build");
#endif
}

extern "C" int zs_debug_stamps_wg(zs_handle* h, uint64_t* out, int32_t n_wgs, int32_t n_phase) {
#ifdef ZS_STAMPS
    if (!h || !out || n_wgs < 0 || n_wgs > ZS_STAMP_WGS || n_phase < 1 || n_phase > ZS_NPHASE)
        return fail(ZS_EINVAL, "bad argument");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> buf((size_t)ZS_STAMP_WGS * ZS_NPHASE);
    HIPCHK(stamps_of(h->G, buf.data(), nullptr, 1));
    for (int w = 0; w < n_wgs; w++)
        for (int k = 0; k < n_phase; k++) out[(size_t)w * n_phase + k] = buf[(size_t)w * ZS_NPHASE + k];
    return ZS_OK;
#else
    (void)h; (void)out; (void)n_wgs; (void)n_phase;
    return fail(ZS_ESTATE, "not a ZS_STAMPS diagnostic build");
#endif
}

// per-phase sums over the step-kernel unit of this handle's G and the reset unit (k_reset's phases)
extern "C" int zs_debug_stamps(zs_handle* h, uint64_t* sum_out, uint64_t* max_out, int32_t n) {
#ifdef ZS_STAMPS
    if (!h || !sum_out || n > ZS_NPHASE) return fail(ZS_EINVAL, "bad argument");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned long long> buf((size_t)ZS_STAMP_WGS * ZS_NPHASE), rb(buf.size());
    HIPCHK(stamps_of(h->G, buf.data(), nullptr, 1));
    HIPCHK(stamps_reset(rb.data(), 1));
    for (int k = 0; k < n; k++) {
        sum_out[k] = 0;
        if (max_out) max_out[k] = 0;
    }
    for (size_t w = 0; w < (size_t)ZS_STAMP_WGS; w++)
        for (int k = 0; k < n; k++) {
            unsigned long long v = buf[w * ZS_NPHASE + k] + rb[w * ZS_NPHASE + k];
            sum_out[k] += v;
            if (max_out && v > max_out[k]) max_out[k] = v;
        }
    return ZS_OK;
#else
    (void)h; (void)sum_out; (void)max_out; (void)n;
    return fail(ZS_ESTATE, "not a ZS_STAMPS diagnostic build");
#endif
}
