"""Same-box A/B against a git revision: build libgsamd.so from REV's csrc/ + include/ (plain
build, no diagnostics) into ab_libs/libgsamd_NAME.so for tools/run_ab_bench.sh.
Usage (here, on the CPU):  python tools/ab_git.py NAME REV [--sub FILE OLD NEW ...]
REV "WORKTREE" takes the working tree; each --sub replaces OLD by NEW (exactly once) in
gymnasium-solver_amd/csrc/FILE before the build (a one-line variant of the current sources).
ab_libs/ is not gpurun-ignored: delete it after the A/B call so later pushes stay small."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gymnasium-solver_amd")]
import build_lib  # noqa: E402

name, rev = sys.argv[1], sys.argv[2]
subs, rest = [], sys.argv[3:]
while rest:
    if rest[0] != "--sub" or len(rest) < 4:
        raise SystemExit("usage: ab_git.py NAME REV [--sub FILE OLD NEW ...]")
    subs.append(tuple(rest[1:4]))
    rest = rest[4:]
tmp = os.path.join("/tmp", f"abrev_{name}")
shutil.rmtree(tmp, ignore_errors=True)
os.makedirs(tmp)
if rev == "WORKTREE":
    for d in ("gymnasium-solver_amd/csrc", "include"):
        shutil.copytree(os.path.join(ROOT, d), os.path.join(tmp, d))
else:
    arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "gymnasium-solver_amd/csrc", "include"],
                          check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
csrc = os.path.join(tmp, "gymnasium-solver_amd", "csrc")
for f, old, new in subs:
    path = os.path.join(csrc, f)
    text = open(path).read()
    if text.count(old) != 1:
        raise SystemExit(f"--sub: {old!r} occurs {text.count(old)} times in {f}")
    open(path, "w").write(text.replace(old, new))
bdir = os.path.join(tmp, "build")
os.makedirs(bdir)
srcs = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".cpp")))
from concurrent.futures import ThreadPoolExecutor  # noqa: E402
with ThreadPoolExecutor(8) as ex:
    list(ex.map(lambda s: build_lib._compile(s, bdir, (), csrc), srcs))
os.makedirs(os.path.join(ROOT, "ab_libs"), exist_ok=True)
out = os.path.join(ROOT, "ab_libs", f"libgsamd_{name}.so")
cmd = [build_lib.HIPCC, f"--offload-arch={build_lib.ARCH}", "-shared", "-fPIC", "-o", out] + \
    [os.path.join(bdir, s + ".o") for s in srcs] + ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
subprocess.run(cmd, check=True)
print("built", out)
