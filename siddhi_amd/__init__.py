"""siddhi_amd: Siddhi's filtered windowed group-by aggregation path on MI355X (gfx950)."""
import ctypes as _C
import os as _os
import warnings as _warnings


def bind_hip_runtime():
    """Keep ONE HIP runtime in the process. libsiddhi_hip.so links the system runtime
    (/opt/rocm/lib/libamdhip64.so.7); PyTorch-ROCm wheels bundle their own libamdhip64.so, which a
    process would otherwise load as a second runtime — and a second runtime initialised after the
    first has enumerated the GPUs finds none ("No HIP GPUs are available"). Loading the system
    runtime under the bare name `libamdhip64.so` before torch makes torch's libraries bind to it.

    Called once at import unless SIDDHI_AMD_BIND_HIP=0 (INTEGRATION.md "Import order"). Returns the
    system runtime's version (hipRuntimeGetVersion), or None when it did nothing: torch was imported
    first (its runtime is already initialised; the two then coexist as before) or no system runtime
    is on the loader path. When torch is imported afterwards it runs on the system runtime; a wheel
    built for a different ROCm major version than the system's is warned about."""
    try:
        with open("/proc/self/maps") as f:
            if "torch/lib/libamdhip64.so" in f.read():
                return None
        lib = _C.CDLL("libamdhip64.so", mode=_C.RTLD_GLOBAL)
    except OSError:
        return None
    ver = _C.c_int(0)
    try:
        if lib.hipRuntimeGetVersion(_C.byref(ver)) != 0:
            return None
    except AttributeError:
        return None
    try:  # the wheel's own ROCm major (torch.version.hip is read without initialising torch's runtime)
        import importlib.util
        spec = importlib.util.find_spec("torch")
        vfile = _os.path.join(_os.path.dirname(spec.origin), "version.py") if spec and spec.origin else None
        if vfile and _os.path.exists(vfile):
            import re
            with open(vfile) as f:
                m = re.search(r"^hip\b.*=\s*'([0-9][^']*)'", f.read(), re.M)
            wheel = m.group(1) if m else ""
            major = ver.value // 10_000_000
            if wheel and int(wheel.split(".")[0]) != major:
                _warnings.warn(f"siddhi_amd binds the system HIP runtime (major {major}) for a torch wheel built "
                               f"for HIP {wheel}; set SIDDHI_AMD_BIND_HIP=0 to keep torch's bundled runtime")
    except Exception:  # version probing is advisory only
        pass
    return ver.value


if _os.environ.get("SIDDHI_AMD_BIND_HIP", "1") != "0":
    bind_hip_runtime()
