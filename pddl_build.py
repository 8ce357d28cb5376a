"""Build the native extensions in-tree for gfx950 (hipcc for the kernels) and place them next to the package.

    python pddl_build.py            # hipcc cross-compiles; no GPU needed
"""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "parallel-and-distributed-deep-learning_amd")


def _check_undefined(so):
    """Fail the build if any pddl symbol (e.g. a kernel's host launch stub) stayed undefined:
    the dynamic loader would only report it at import time on the GPU box."""
    r = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True)
    bad = [ln.split()[-1] for ln in r.stdout.splitlines() if "4pddl" in ln]
    if bad:
        raise RuntimeError(f"{os.path.basename(so)} has undefined pddl symbols: {bad[:4]}")


def build(verbose: bool = False) -> str:
    env = dict(os.environ)
    env.setdefault("PDDL_OFFLOAD_ARCH", "gfx950")
    env.setdefault("MAX_JOBS", "8")
    # object files stay outside the tree so GPU-box snapshots only carry the .so files
    cmd = [sys.executable, "setup.py", "build_ext", "--inplace", "--build-temp",
           os.path.join(os.environ.get("TMPDIR", "/tmp"), "pddl_build_temp")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=not verbose, text=True)
    shutil.rmtree(os.path.join(ROOT, "build"), ignore_errors=True)
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "")[-4000:] + (r.stderr or "")[-4000:])
        raise RuntimeError("native build failed")
    out = []
    for name in ("_pddl_native", "_pddl_h5", "_pddl_io"):
        built = sorted(glob.glob(os.path.join(ROOT, f"{name}*.so")))
        if not built:
            raise RuntimeError(f"native build produced no {name} shared object")
        dst = os.path.join(PKG, os.path.basename(built[-1]))
        shutil.move(built[-1], dst)
        _check_undefined(dst)
        out.append(dst)
    return out[0]


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
