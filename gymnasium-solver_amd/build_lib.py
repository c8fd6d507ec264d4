"""Build libgsamd.so (HIP for gfx950 + host C++) in-tree with plain hipcc command lines.

Objects go to gymnasium-solver_amd/build/, the library to gymnasium-solver_amd/gsamd/libgsamd.so
(git-ignored; it travels to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "gsamd", "libgsamd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

# per-file extra flags: the GAE scan must not contract mul+add into FMA (bit-exactness
# with the reference's numpy float32 loop)
EXTRA = {"gs_gae.hip": ["-ffp-contract=off"], "gs_mlp.hip": ["-ffp-contract=off"], "gs_atari.hip": ["-ffp-contract=off"],
         "gs_cartpole.hip": ["-ffp-contract=off"]}


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _obj(src):
    return os.path.join(BUILD, src + ".o")


def _source_hashes(csrc=None):
    """gsamd/buildinfo.source_hash of the measured paths, embedded into gs_abi.cpp
    (gs_build_source_hash) so a measurement can be tied to the loaded binary."""
    sys.path.insert(0, os.path.join(HERE, "gsamd"))
    try:
        import buildinfo
    finally:
        sys.path.pop(0)
    kw = {"csrc": csrc} if csrc else {}
    return {"MLP": buildinfo.source_hash("mlp", **kw), "CNN": buildinfo.source_hash("cnn", **kw),
            "ALL": buildinfo.source_hash(None, **kw)}


def _compile(src, build_dir=None, defines=(), csrc=None, hashes=None):
    csrc = csrc or CSRC
    path = os.path.join(csrc, src)
    obj = os.path.join(build_dir, src + ".o") if build_dir else _obj(src)
    deps = [path, os.path.join(HERE, "..", "include", "gsamd.h")] + [
        os.path.join(csrc, h) for h in os.listdir(csrc) if h.endswith(".h")]
    hdefs = []
    if src == "gs_abi.cpp" and hashes:
        hdefs = [f'-DGS_SRC_HASH_{k}="{v}"' for k, v in sorted(hashes.items())]
        stamp = obj + ".hash"
        if not os.path.exists(stamp) or open(stamp).read() != " ".join(hdefs):
            if os.path.exists(obj):
                os.remove(obj)
            with open(stamp, "w") as f:
                f.write(" ".join(hdefs))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return None
    cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-c", path, "-o", obj]
    if src.endswith(".hip"):
        cmd[1:1] = [f"--offload-arch={ARCH}", "-x", "hip"]
    cmd += EXTRA.get(src, []) + [f"-D{d}" for d in defines] + hdefs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return src


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    hashes = _source_hashes()
    with ThreadPoolExecutor(max_workers=min(jobs, len(srcs))) as ex:
        done = [s for s in ex.map(lambda s: _compile(s, hashes=hashes), srcs) if s]
    objs = [_obj(s) for s in srcs]
    if done or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + [
            "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB} ({len(done)} objects recompiled)")
    return LIB


def build_variant(out_path: str, defines, jobs: int = 8, patches=(), tag: str = "") -> str:
    """Diagnostic variant (e.g. GS_STAMPS phase timers) built into its own directory.  patches:
    (file, old, new) source substitutions applied to a copy of csrc/ (timing experiments live in
    tools/ab_experiments.py, not in the product sources)."""
    import shutil
    bdir = os.path.join(BUILD, "variant_" + "_".join(list(defines) + ([tag] if tag else [])))
    os.makedirs(bdir, exist_ok=True)
    csrc = None
    if patches:
        # bdir/src/csrc: its sources' "../../include/gsamd.h" resolves to bdir/include -> include/
        csrc = os.path.join(bdir, "src", "csrc")
        shutil.rmtree(os.path.dirname(csrc), ignore_errors=True)
        shutil.copytree(CSRC, csrc)
        inc = os.path.join(bdir, "include")
        if not os.path.exists(inc):
            os.symlink(os.path.join(HERE, "..", "include"), inc)
        for f, old, new in patches:
            fp = os.path.join(csrc, f)
            text = open(fp).read()
            if old not in text:
                raise RuntimeError(f"experiment patch does not apply to {f}: {old[:60]!r}...")
            open(fp, "w").write(text.replace(old, new))
    srcs = _sources()
    with ThreadPoolExecutor(max_workers=min(jobs, len(srcs))) as ex:
        list(ex.map(lambda s: _compile(s, bdir, defines, csrc, hashes=_source_hashes(csrc)), srcs))
    objs = [os.path.join(bdir, s + ".o") for s in srcs]
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out_path] + objs + [
        "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return out_path


if __name__ == "__main__":
    build(verbose=True, jobs=int(sys.argv[1]) if len(sys.argv) > 1 else 8)
