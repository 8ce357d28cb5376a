"""Loader for the in-tree native extension `_pddl_native` (HIP kernels for gfx950).

The shared object is built by ``python pddl_build.py`` (or ``__graft_entry__.build()``) and
lives next to this package.  On a GPU machine the GPU path REQUIRES it: `require_native()`
raises instead of falling back to eager PyTorch, so a test that passes on the GPU has run
the hand-written kernels.
"""
import glob
import importlib.machinery
import importlib.util
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_REPO = os.path.dirname(_PKG)
_native = None
_err = None


def _candidates():
    pats = ["_pddl_native*.so"]
    out = []
    override = os.environ.get("PDDL_NATIVE_DIR")   # e.g. the sanitizer build (scripts/sanitize_host.sh)
    if override:
        return sorted(glob.glob(os.path.join(override, pats[0])))
    for d in (_PKG, _REPO):
        for p in pats:
            out += sorted(glob.glob(os.path.join(d, p)))
    return out


def _load():
    global _native, _err
    if _native is not None or _err is not None:
        return _native
    import torch  # noqa: F401  (libtorch must be loaded first)
    for path in _candidates():
        try:
            loader = importlib.machinery.ExtensionFileLoader("_pddl_native", path)
            spec = importlib.util.spec_from_file_location("_pddl_native", path, loader=loader)
            mod = importlib.util.module_from_spec(spec)
            loader.exec_module(mod)
            sys.modules["_pddl_native"] = mod
            _native = mod
            _apply_knobs(mod)
            return mod
        except Exception as e:  # pragma: no cover - reported by require_native
            _err = f"{path}: {e}"
    if _err is None:
        _err = "no _pddl_native*.so found (run `python pddl_build.py`)"
    return None


def _apply_knobs(mod):
    """PDDL_KNOBS="igemm8=1,igemm_pk=0": kernel tuning knobs for A/B runs of whole
    programs (bench.py, the entry scripts) without code changes."""
    spec = os.environ.get("PDDL_KNOBS", "").strip()
    for item in filter(None, (x.strip() for x in spec.split(","))):
        name, _, val = item.partition("=")
        mod.set_variant(name.strip(), int(val))


def native_available() -> bool:
    return _load() is not None


def require_native():
    mod = _load()
    if mod is None:
        raise RuntimeError(f"pddl native HIP extension unavailable: {_err}")
    return mod


class _Proxy:
    def __getattr__(self, name):
        return getattr(require_native(), name)


native = _Proxy()
