"""ORACLE — test infrastructure only (CPU restatement of the reference's hot path).

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker.  The product path (gymnasium-solver_amd/) never imports anything here;
tests/test_host_cpu.py::test_product_does_not_import_oracle enforces that.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build(verbose=False):
    """Compile the C/C++ restatements into oracle/_build/liboracle.so (gcc/g++ only)."""
    import subprocess
    os.makedirs(os.path.join(_HERE, "_build"), exist_ok=True)
    objs = []
    for src, cc in (("gae_ref.c", "gcc"), ("sampler_ref.cpp", "g++")):
        obj = os.path.join(_HERE, "_build", src + ".o")
        cmd = [cc, "-O2", "-fPIC", "-ffp-contract=off", "-c", os.path.join(_HERE, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        objs.append(obj)
    subprocess.check_call(["g++", "-shared", "-o", LIB_PATH] + objs)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, f64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
        L.oracle_gae_f32.argtypes = [vp, vp, vp, vp, vp, vp, i64, i64, f64, f64, vp, vp]
        L.oracle_gae_f32.restype = None
        L.oracle_sampler_stream.argtypes = [i64, i64, ctypes.c_uint64, vp]
        L.oracle_sampler_stream.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def gae_c(values, rewards, dones, timeouts, last_values, bootstrap, gamma, lam):
    values = np.ascontiguousarray(values, np.float32)
    T, N = values.shape
    rewards = np.ascontiguousarray(rewards, np.float32)
    dones = np.ascontiguousarray(dones, np.uint8)
    timeouts = np.ascontiguousarray(timeouts, np.uint8)
    last_values = np.ascontiguousarray(last_values, np.float32)
    bootstrap = None if bootstrap is None else np.ascontiguousarray(bootstrap, np.float32)
    adv = np.empty((T, N), np.float32)
    ret = np.empty((T, N), np.float32)
    lib().oracle_gae_f32(_p(values), _p(rewards), _p(dones), _p(timeouts), _p(bootstrap), _p(last_values),
                         T, N, float(gamma), float(lam), _p(adv), _p(ret))
    return adv, ret


def sampler_stream(data_len, num_passes, seed):
    out = np.empty(int(data_len) * int(num_passes), np.int64)
    lib().oracle_sampler_stream(int(data_len), int(num_passes), int(seed), _p(out))
    return out
