"""Loader of the in-tree HIP library (crocoddyl_amd/lib/libfddp_hip.so).

There is no CPU fallback: if the library is missing or no gfx950 device is
usable, every solver entry point raises. Build it with
``python -c "import __graft_entry__ as g; g.build()"`` or ``make -C crocoddyl_amd/csrc``.
"""
import ctypes as C
import os

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CROCODDYL_AMD_LIB") or os.path.join(_HERE, "lib", "libfddp_hip.so")

_lib = None


class FDDPError(RuntimeError):
    """Raised for argument errors (the reference's throw_pretty) and runtime failures."""


def _share_torch_hip_runtime():
    """A process may hold only one HIP runtime. PyTorch-ROCm wheels bundle
    their own libamdhip64 (same soname, different file); if torch is
    installed, load that one first (RTLD_GLOBAL) so libfddp_hip binds to it
    and torch and this library share one runtime in either import order."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            C.CDLL(p, mode=C.RTLD_GLOBAL)
            return


def lib():
    global _lib
    if _lib is None:
        _share_torch_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"crocoddyl_amd: HIP library not built ({LIB_PATH} missing); "
                              "run __graft_entry__.build() — there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        _abi.bind(L, "fddp_", _abi.PROTOS)
        _abi.bind(L, "fddp_", _abi.PROTOS_GPU)
        v = L.fddp_abi_version()
        if v != _abi.ABI_VERSION:
            raise ImportError(f"crocoddyl_amd: {LIB_PATH} has C ABI version {v}, this binding needs "
                              f"{_abi.ABI_VERSION} (rebuild it)")
        _lib = L
    return _lib


def check(rc):
    if rc != _abi.FDDP_OK:
        msg = lib().fddp_last_error().decode(errors="replace")
        raise FDDPError(f"libfddp_hip error {rc}: {msg}")
    return rc


def default_params():
    p = _abi.Params()
    lib().fddp_default_params(C.byref(p))
    return p
