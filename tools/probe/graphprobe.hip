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
