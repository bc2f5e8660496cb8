import ctypes, os, re, sys
here = os.path.dirname(os.path.abspath(__file__))
mode = sys.argv[1]
def libs():
    return sorted(set(re.findall(r'\S*(?:amdhip64|hsa-runtime64)\S*', open('/proc/self/maps').read())))
def run(so):
    L = ctypes.CDLL(os.path.join(here, so)); m = ctypes.create_string_buffer(256)
    rc = L.probe_run(m, 256); print(mode, so, "rc=", rc, m.value.decode(), libs(), flush=True)
if mode == "notorch":
    run("probe.so")
elif mode == "torch_first":
    import torch; x = torch.zeros(1, device="cuda"); print("torch hip", torch.version.hip, x.device, flush=True)
    run("probe.so"); run("probe_nocomp.so")
elif mode == "preload":
    ctypes.CDLL("/opt/rocm/lib/libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    run("probe.so")
    import torch; x = torch.ones(4, device="cuda") * 2; print("torch after preload ok", x.sum().item(), libs(), flush=True)
