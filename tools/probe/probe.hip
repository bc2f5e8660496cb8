// HIP runtime probe: which runtime is loaded, does a device show up, does a gfx950 kernel launch.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_probe(int* out) { out[threadIdx.x] = threadIdx.x * 3 + 1; }
extern "C" int probe_run(char* msg, int len) {
    int n = -1;
    hipError_t e = hipGetDeviceCount(&n);
    int rtv = 0; hipRuntimeGetVersion(&rtv);
    if (e != hipSuccess) { snprintf(msg, len, "hipGetDeviceCount: %s (rt %d)", hipGetErrorString(e), rtv); return 1; }
    e = hipSetDevice(0);
    if (e != hipSuccess) { snprintf(msg, len, "hipSetDevice: %s (n=%d rt %d)", hipGetErrorString(e), n, rtv); return 2; }
    int* d = nullptr; e = hipMalloc(&d, 256);
    if (e != hipSuccess) { snprintf(msg, len, "hipMalloc: %s", hipGetErrorString(e)); return 3; }
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d);
    e = hipGetLastError();
    if (e != hipSuccess) { snprintf(msg, len, "launch: %s", hipGetErrorString(e)); return 4; }
    int h[64]; e = hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    if (e != hipSuccess) { snprintf(msg, len, "memcpy: %s", hipGetErrorString(e)); return 5; }
    hipFree(d);
    snprintf(msg, len, "ok n=%d rt=%d out[5]=%d", n, rtv, h[5]);
    return h[5] == 16 ? 0 : 6;
}
#ifdef PROBE_MAIN
int main() { char m[256]; int rc = probe_run(m, 256); printf("exe: rc=%d %s\n", rc, m); return rc; }
#endif
