"""siddhi_amd: Siddhi's filtered windowed group-by aggregation path on MI355X (gfx950)."""
import ctypes as _C


def _bind_hip_runtime():
    """Keep ONE HIP runtime in the process. libsiddhi_hip.so links the system runtime
    (/opt/rocm/lib/libamdhip64.so.7); PyTorch-ROCm wheels bundle their own libamdhip64.so, which a
    process would otherwise load as a second runtime — and a second runtime initialised after the
    first has enumerated the GPUs finds none ("No HIP GPUs are available"). Loading the system
    runtime under the bare name `libamdhip64.so` before torch makes torch's libraries bind to it.
    When torch was imported first its runtime is already initialised and this is a no-op."""
    try:
        with open("/proc/self/maps") as f:
            if "torch/lib/libamdhip64.so" in f.read():
                return
        _C.CDLL("libamdhip64.so", mode=_C.RTLD_GLOBAL)
    except OSError:
        pass


_bind_hip_runtime()
