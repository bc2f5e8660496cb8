// Does a captured hipGraph deliver kernel arguments and small memsets intact?  (diagnostic only)
// Kernels here never dereference an argument: each writes a checksum of its by-value argument
// bytes into a sentinel buffer, launched directly and through a captured graph, and the two are
// compared; a 4-byte memset is captured into a graph and the neighbouring words checked.
// hipcc --offload-arch=gfx950 -O3 -o graphprobe tools/probe/graphprobe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int NW>
struct Big {
    uint32_t w[NW];
};

__device__ uint32_t g_out[2];  // results go to a global symbol: no argument is ever dereferenced

template <int NW>
__global__ void k_sum(Big<NW> b, int tail) {
    if (threadIdx.x || blockIdx.x) return;
    uint32_t s = 0;
    for (int i = 0; i < NW; i++) s = s * 31u + b.w[i];
    g_out[0] = s;
    g_out[1] = (uint32_t)tail;
}

// dynamic LDS: write a pattern over the whole requested size, read it back, report the mismatches
__global__ void k_lds(int bytes) {
    extern __shared__ uint32_t lds[];
    const int n = bytes / 4;
    for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = 0x5a5a0000u ^ (uint32_t)i;
    __syncthreads();
    int bad = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) bad += lds[i] != (0x5a5a0000u ^ (uint32_t)i);
    atomicAdd(&g_out[0], (uint32_t)bad);
    if (threadIdx.x == 0) atomicAdd(&g_out[1], 1u);
}

int probe_lds(hipStream_t s, int bytes) {
    const uint32_t zero[2] = {0, 0};
    uint32_t direct[2], graph[2];
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), zero, 8));
    hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), bytes, s, bytes);
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpyFromSymbol(direct, HIP_SYMBOL(g_out), 8));
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), zero, 8));
    hipStream_t cs;
    CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t x;
    CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), bytes, cs, bytes);
    CHK(hipStreamEndCapture(cs, &g));
    CHK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(x, s));
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpyFromSymbol(graph, HIP_SYMBOL(g_out), 8));
    printf("dynamic LDS %6d B: direct bad=%u runs=%u  graph bad=%u runs=%u  %s\n", bytes, direct[0], direct[1], graph[0],
           graph[1], direct[0] == 0 && graph[0] == 0 && graph[1] == 1 ? "OK" : "MISMATCH");
    CHK(hipGraphExecDestroy(x));
    CHK(hipGraphDestroy(g));
    CHK(hipStreamDestroy(cs));
    return 0;
}

template <int NW>
int probe(hipStream_t s) {
    Big<NW> b;
    for (int i = 0; i < NW; i++) b.w[i] = 0x9e3779b9u * (i + 1);
    uint32_t direct[2] = {0, 0}, graph[2] = {0, 0};
    const uint32_t zero[2] = {0, 0};
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), zero, 8));
    hipLaunchKernelGGL(k_sum<NW>, dim3(1), dim3(64), 0, s, b, 12345);
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpyFromSymbol(direct, HIP_SYMBOL(g_out), 8));
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), zero, 8));
    hipStream_t cs;
    CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t x;
    CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k_sum<NW>, dim3(1), dim3(64), 0, cs, b, 12345);
    CHK(hipStreamEndCapture(cs, &g));
    CHK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(x, s));
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpyFromSymbol(graph, HIP_SYMBOL(g_out), 8));
    printf("args %4d B: direct %08x/%u  graph %08x/%u  %s\n", (int)sizeof(b) + 12, direct[0], direct[1], graph[0],
           graph[1], direct[0] == graph[0] && direct[1] == graph[1] ? "OK" : "MISMATCH");
    CHK(hipGraphExecDestroy(x));
    CHK(hipGraphDestroy(g));
    CHK(hipStreamDestroy(cs));
    return 0;
}

// The engine's form: per pending-list parity q a graph zeroes counter cnt[q] with a captured 4-byte
// hipMemsetAsync, then a kernel appends to it (atomicAdd from 64 lanes, the returned maximum recorded
// per replay).  The two graphs are captured on one non-blocking stream and replayed alternately; a
// correct replay leaves exactly 64 in cnt[q].  No address is ever derived from a counter value.
__global__ void k_append(int* cnt, int* rec, int replay) {
    const int v = atomicAdd(cnt, 1);
    atomicMax(&rec[replay], v + 1);
}

int probe_chain(hipStream_t s, int replays, int lds) {
    int *cnt, *rec;
    CHK(hipMalloc(&cnt, 16));  // the engine's minimum allocation for d_rcount[2]
    CHK(hipMemset(cnt, 0, 16));
    CHK(hipMalloc(&rec, sizeof(int) * replays));
    CHK(hipMemset(rec, 0, sizeof(int) * replays));
    hipStream_t cs;
    CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraphExec_t x[2];
    for (int q = 0; q < 2; q++) {
        hipGraph_t g;
        CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        CHK(hipMemsetAsync(cnt + q, 0, sizeof(int), cs));
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), lds, cs, lds);  // a kernel with dynamic LDS between
        hipLaunchKernelGGL(k_append, dim3(1), dim3(64), 0, cs, cnt + q, rec, 0);
        CHK(hipStreamEndCapture(cs, &g));
        CHK(hipGraphInstantiate(&x[q], g, nullptr, nullptr, 0));
        CHK(hipGraphDestroy(g));
    }
    // replay: graph q each time, the recorded maximum per replay goes to rec[0]; read it back per replay
    int bad = 0, first_bad = -1, worst = 0;
    for (int i = 0; i < replays; i++) {
        CHK(hipMemsetAsync(rec, 0, sizeof(int), s));
        CHK(hipGraphLaunch(x[i & 1], s));
        int got = 0;
        CHK(hipMemcpyAsync(&got, rec, sizeof(int), hipMemcpyDeviceToHost, s));
        CHK(hipStreamSynchronize(s));
        if (got != 64) {
            bad++;
            if (first_bad < 0) first_bad = i;
            worst = got > worst ? got : worst;
        }
    }
    int host[4] = {0, 0, 0, 0};
    CHK(hipMemcpy(host, cnt, 16, hipMemcpyDeviceToHost));
    printf("memset+append chain, %d replays, %d B LDS between: %d bad (first %d, worst count %d), counters %d %d %d %d  %s\n",
           replays, lds, bad, first_bad, worst, host[0], host[1], host[2], host[3], bad ? "MISMATCH" : "OK");
    for (int q = 0; q < 2; q++) CHK(hipGraphExecDestroy(x[q]));
    CHK(hipStreamDestroy(cs));
    CHK(hipFree(cnt));
    CHK(hipFree(rec));
    return 0;
}

// The deferred-respawn form: two captured 4-byte memsets in a row (the parity's list counter, then a
// second counter in its own allocation), then a kernel appending to both.
__global__ void k_append2(int* c1, int* c2, int* rec) {
    const int v = atomicAdd(c1, 1), w = atomicAdd(c2, 1);
    atomicMax(&rec[0], v + 1);
    atomicMax(&rec[1], w + 1);
}

// fills the host stack below the caller with a byte pattern (the frames the capture calls used)
__attribute__((noinline)) void scribble_stack(unsigned char pat) {
    volatile unsigned char buf[256 * 1024];
    for (size_t i = 0; i < sizeof(buf); i++) buf[i] = pat;
}

// memset nodes followed by a kernel whose by-value argument block is large (the engine's Dev struct
// is ~0.4 KB): are the kernel's arguments intact when the graph replays?
template <int NW>
int probe_memset_args(hipStream_t s, int n_memsets) {
    Big<NW> b;
    for (int i = 0; i < NW; i++) b.w[i] = 0x9e3779b9u * (i + 7);
    const uint32_t zero[2] = {0, 0};
    uint32_t direct[2], graph[2];
    int* cnt;
    CHK(hipMalloc(&cnt, 16));
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), zero, 8));
    hipLaunchKernelGGL(k_sum<NW>, dim3(1), dim3(64), 0, s, b, 777);
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpyFromSymbol(direct, HIP_SYMBOL(g_out), 8));
    hipStream_t cs;
    CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t x;
    CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    for (int m = 0; m < n_memsets; m++) CHK(hipMemsetAsync(cnt + m, 0, sizeof(int), cs));
    hipLaunchKernelGGL(k_sum<NW>, dim3(1), dim3(64), 0, cs, b, 777);
    CHK(hipStreamEndCapture(cs, &g));
    CHK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    int bad = 0;
    for (int rep = 0; rep < 20; rep++) {
        CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), zero, 8));
        CHK(hipGraphLaunch(x, s));
        CHK(hipStreamSynchronize(s));
        CHK(hipMemcpyFromSymbol(graph, HIP_SYMBOL(g_out), 8));
        bad += graph[0] != direct[0] || graph[1] != direct[1];
    }
    printf("%d memset node(s) then a kernel with %4d B of arguments: %d of 20 replays with other arguments  %s\n",
           n_memsets, (int)sizeof(b) + 4, bad, bad ? "MISMATCH" : "OK");
    CHK(hipGraphExecDestroy(x));
    CHK(hipGraphDestroy(g));
    CHK(hipStreamDestroy(cs));
    CHK(hipFree(cnt));
    return 0;
}

int probe_chain2(hipStream_t s, int replays, int kernel_between, int scribble = 0) {
    int *cnt, *resp, *rec;
    CHK(hipMalloc(&cnt, 16));
    CHK(hipMalloc(&resp, 16));
    CHK(hipMemset(cnt, 0, 16));
    CHK(hipMemset(resp, 0, 16));
    CHK(hipMalloc(&rec, 2 * sizeof(int)));
    hipStream_t cs;
    CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraphExec_t x[2];
    for (int q = 0; q < 2; q++) {
        hipGraph_t g;
        CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        if (kernel_between) hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 1024, cs, 1024);
        CHK(hipMemsetAsync(cnt + q, 0, sizeof(int), cs));
        CHK(hipMemsetAsync(resp, 0, sizeof(int), cs));
        if (scribble > 1) scribble_stack((unsigned char)(0x50 + q));  // dirty the stack before the rest of the capture
        hipLaunchKernelGGL(k_append2, dim3(1), dim3(64), 0, cs, cnt + q, resp, rec);
        CHK(hipStreamEndCapture(cs, &g));
        if (scribble > 1) scribble_stack((unsigned char)(0x60 + q));  // ... and before instantiation
        CHK(hipGraphInstantiate(&x[q], g, nullptr, nullptr, 0));
        CHK(hipGraphDestroy(g));
    }
    int bad = 0, first_bad = -1, w1 = 0, w2 = 0;
    for (int i = 0; i < replays; i++) {
        if (scribble) scribble_stack((unsigned char)(0x40 + (i & 1)));
        CHK(hipMemsetAsync(rec, 0, 2 * sizeof(int), s));
        CHK(hipGraphLaunch(x[i & 1], s));
        int got[2] = {0, 0};
        CHK(hipMemcpyAsync(got, rec, sizeof(got), hipMemcpyDeviceToHost, s));
        CHK(hipStreamSynchronize(s));
        if (got[0] != 64 || got[1] != 64) {
            bad++;
            if (first_bad < 0) first_bad = i;
            w1 = got[0] > w1 ? got[0] : w1;
            w2 = got[1] > w2 ? got[1] : w2;
        }
    }
    printf("two memsets + append, %d replays, kernel before: %d, host stack overwritten (1: between replays, "
           "2: also during capture and before instantiation): %d: %d bad (first %d, worst counts 0x%08x 0x%08x)  %s\n",
           replays, kernel_between, scribble, bad,
           first_bad, w1, w2, bad ? "MISMATCH" : "OK");
    for (int q = 0; q < 2; q++) CHK(hipGraphExecDestroy(x[q]));
    CHK(hipStreamDestroy(cs));
    CHK(hipFree(cnt));
    CHK(hipFree(resp));
    CHK(hipFree(rec));
    return 0;
}

// The engine's city128 step graph as it was captured with ZS_GRAPH_MEMSET=1 (round 2), node for node:
// on the capture stream an event record (the reset fork), the policy kernel, then on a side stream
// (waiting on that event) a one-wave kernel with dynamic LDS (k_reset), its join event; back on the
// capture stream the two captured 4-byte memsets (the parity's pending-list counter, then the
// deferred-respawn counter in its own allocation), the step kernel (one-wave workgroups, a by-value
// argument block of the engine's Dev size, dynamic LDS) appending to both counters, the respawn kernel
// (appends nothing), the wait on the join, and the observation kernel.  Two graphs (one per list
// parity) replayed alternately; a correct replay leaves exactly `waves` in both counters.
template <int NW>
__global__ void k_step_like(Big<NW> b, int* c1, int* c2, int* rec, int bytes) {
    extern __shared__ uint32_t lds[];
    for (int i = threadIdx.x; i < bytes / 4; i += 64) lds[i] = b.w[i % NW] ^ (uint32_t)i;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int v = atomicAdd(c1, 1), w = atomicAdd(c2, 1);
        atomicMax(&rec[0], v + 1);
        atomicMax(&rec[1], w + 1);
    }
}

template <int NW>
__global__ void k_other(Big<NW> b, int bytes) {
    extern __shared__ uint32_t lds[];
    for (int i = threadIdx.x; i < bytes / 4; i += 64) lds[i] = b.w[i % NW];
    __syncthreads();
    if (threadIdx.x == 0 && lds[0] == 0xdeadbeefu) g_out[0] = 1;
}

int probe_fork(hipStream_t s, int replays, int waves) {
    constexpr int NW = 180;  // 720 B by value, about the engine's Dev
    Big<NW> b;
    for (int i = 0; i < NW; i++) b.w[i] = 0x9e3779b9u * (i + 3);
    int *cnt, *resp, *rec;
    CHK(hipMalloc(&cnt, 16));
    CHK(hipMalloc(&resp, 16));
    CHK(hipMemset(cnt, 0, 16));
    CHK(hipMemset(resp, 0, 16));
    CHK(hipMalloc(&rec, 2 * sizeof(int)));
    hipStream_t cs, side;
    CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CHK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CHK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    hipGraphExec_t x[2];
    for (int q = 0; q < 2; q++) {
        hipGraph_t g;
        CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        CHK(hipEventRecord(fork, cs));
        hipLaunchKernelGGL(k_other<NW>, dim3(64), dim3(64), 0, cs, b, 0);               // policy
        CHK(hipStreamWaitEvent(side, fork, 0));
        hipLaunchKernelGGL(k_other<NW>, dim3(256), dim3(64), 20480, side, b, 20480);    // reset, side stream
        CHK(hipEventRecord(join, side));
        CHK(hipMemsetAsync(cnt + (1 - q), 0, sizeof(int), cs));                         // list counter
        CHK(hipMemsetAsync(resp, 0, sizeof(int), cs));                                  // respawn counter
        hipLaunchKernelGGL(k_step_like<NW>, dim3(waves), dim3(64), 24576, cs, b, cnt + (1 - q), resp, rec, 24576);
        hipLaunchKernelGGL(k_other<NW>, dim3(512), dim3(64), 20480, cs, b, 20480);      // respawn
        CHK(hipStreamWaitEvent(cs, join, 0));
        hipLaunchKernelGGL(k_other<NW>, dim3(1024), dim3(256), 16384, cs, b, 16384);    // observations
        CHK(hipStreamEndCapture(cs, &g));
        CHK(hipGraphInstantiate(&x[q], g, nullptr, nullptr, 0));
        CHK(hipGraphDestroy(g));
    }
    int bad = 0, first_bad = -1;
    unsigned w1 = 0, w2 = 0;
    for (int i = 0; i < replays; i++) {
        CHK(hipMemsetAsync(rec, 0, 2 * sizeof(int), s));
        CHK(hipGraphLaunch(x[i & 1], s));
        int got[2] = {0, 0};
        CHK(hipMemcpyAsync(got, rec, sizeof(got), hipMemcpyDeviceToHost, s));
        CHK(hipStreamSynchronize(s));
        if (got[0] != waves || got[1] != waves) {
            bad++;
            if (first_bad < 0) first_bad = i;
            w1 = (unsigned)got[0] > w1 ? (unsigned)got[0] : w1;
            w2 = (unsigned)got[1] > w2 ? (unsigned)got[1] : w2;
        }
    }
    printf("engine city128 graph shape (fork/join, 2 memsets, %d-workgroup append), %d replays: %d bad (first %d, "
           "worst counts 0x%08x 0x%08x)  %s\n",
           waves, replays, bad, first_bad, w1, w2, bad ? "MISMATCH" : "OK");
    for (int q = 0; q < 2; q++) CHK(hipGraphExecDestroy(x[q]));
    CHK(hipEventDestroy(fork));
    CHK(hipEventDestroy(join));
    CHK(hipStreamDestroy(cs));
    CHK(hipStreamDestroy(side));
    CHK(hipFree(cnt));
    CHK(hipFree(resp));
    CHK(hipFree(rec));
    return 0;
}

int main(int argc, char** argv) {
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    uint32_t* buf;
    CHK(hipMalloc(&buf, 64 * sizeof(uint32_t)));
    if (probe<16>(s) || probe<64>(s) || probe<110>(s) || probe<125>(s) || probe<126>(s) ||
        probe<127>(s) || probe<128>(s) || probe<140>(s) || probe<200>(s) || probe<256>(s) ||
        probe<500>(s))
        return 1;
    if (probe_lds(s, 1024) || probe_lds(s, 7744) || probe_lds(s, 14304) || probe_lds(s, 32768) || probe_lds(s, 65536))
        return 1;
    if (argc < 2) return 0;  // "memset": also the captured memset (writes device memory from graph params)
    if (argc > 2) return probe_fork(s, 400, 1) || probe_fork(s, 400, 4096);  // "memset fork": the engine's shape only
    if (probe_chain(s, 200, 1024) || probe_chain(s, 200, 14304)) return 1;
    if (probe_chain2(s, 200, 0) || probe_chain2(s, 200, 1) || probe_chain2(s, 50, 1, 1) || probe_chain2(s, 50, 1, 2))
        return 1;
    if (probe_memset_args<16>(s, 1) || probe_memset_args<100>(s, 1) || probe_memset_args<100>(s, 2) ||
        probe_memset_args<128>(s, 2) || probe_memset_args<200>(s, 2))
        return 1;
    // captured 4-byte memset inside a 16-word sentinel buffer
    uint32_t host[16];
    for (int i = 0; i < 16; i++) host[i] = 0xabababab;
    CHK(hipMemcpy(buf, host, sizeof(host), hipMemcpyHostToDevice));
    hipStream_t cs;
    CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t x;
    CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    CHK(hipMemsetAsync(buf + 5, 0, sizeof(uint32_t), cs));
    CHK(hipStreamEndCapture(cs, &g));
    CHK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(x, s));
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpy(host, buf, sizeof(host), hipMemcpyDeviceToHost));
    int ok = 1;
    for (int i = 0; i < 16; i++) ok &= host[i] == (i == 5 ? 0u : 0xababababu);
    printf("memset 4 B in graph: %s\n", ok ? "OK" : "MISMATCH");
    return 0;
}
