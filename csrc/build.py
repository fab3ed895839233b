#!/usr/bin/env python
"""Build the HIP/CDNA4 kernel library for gfx950.

Every ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950 -O3`` into
an object, then linked into ``speakingstyle_amd/_lib/libssamd_kernels.so`` (the
in-tree location the Python bindings load; the .so is git-ignored but travels
to the GPU box with the repository snapshot).  ``csrc/host_*.cpp`` form the
native host-runtime library ``libssamd_host.so`` (g++, no GPU code).

Usage: python csrc/build.py [--jobs N] [--debug] [--clean] [--sanitize]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT_DIR = os.path.join(ROOT, "speakingstyle_amd", "_lib")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
KLIB = os.path.join(OUT_DIR, "libssamd_kernels.so")
HLIB = os.path.join(OUT_DIR, "libssamd_host.so")
FLIB = os.path.join(OUT_DIR, "ssamd_fast" + sysconfig.get_config_var("EXT_SUFFIX"))  # launch bindings
ARCH = os.environ.get("SSAMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed: %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(jobs=8, debug=False, clean=False, verbose=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    headers = glob.glob(os.path.join(HERE, "*.h"))
    srcs = sorted(glob.glob(os.path.join(HERE, "*.hip")))
    opt = ["-O1", "-g"] if debug else ["-O3"]
    flags = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             "-Wno-unused-variable", "-munsafe-fp-atomics", "-I", HERE] + opt

    def compile_one(src):
        obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
        if clean or _stale(obj, [src] + headers):
            _run([HIPCC, "-c", src, "-o", obj] + flags)
        return obj

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    if clean or _stale(KLIB, objs):
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-Wl,-soname,libssamd_kernels.so", "-o", KLIB] + objs)

    build_fastcall(clean)

    hsrcs = sorted(glob.glob(os.path.join(HERE, "host_*.cpp")))
    if hsrcs and (clean or _stale(HLIB, hsrcs + headers)):
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", HLIB] + hsrcs)
    if verbose:
        print("built", KLIB, FLIB, HLIB if hsrcs else "")
    return KLIB


def build_fastcall(clean=False):
    """Native METH_FASTCALL launch bindings generated from hip._SIGS (csrc/gen_fastcall.py)."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    import gen_fastcall

    src = gen_fastcall.generate(*gen_fastcall.signatures())
    gen_dir = os.path.join(ROOT, "build", "gen")
    os.makedirs(gen_dir, exist_ok=True)
    cpp = os.path.join(gen_dir, "ssamd_fast.cpp")
    old = open(cpp).read() if os.path.exists(cpp) else None
    if old != src:
        with open(cpp, "w") as f:
            f.write(src)
    if clean or _stale(FLIB, [cpp, KLIB]):
        inc = sysconfig.get_paths()["include"]
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", inc, "-o", FLIB, cpp, "-L", OUT_DIR,
              "-l:libssamd_kernels.so", "-Wl,-rpath,$ORIGIN"])
    return FLIB


# Host-only sanitizer builds (GPU sanitizers are not available on the target pool).
SANITIZERS = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
              "tsan": ["-fsanitize=thread"]}


def build_sanitized(verbose=False):
    """Build the host runtime + its self-test (csrc/selftest_host_collate.cpp) under
    ASan+UBSan and under TSan into build/sanitize/; returns {name: executable}."""
    out_dir = os.path.join(ROOT, "build", "sanitize")
    os.makedirs(out_dir, exist_ok=True)
    hsrcs = sorted(glob.glob(os.path.join(HERE, "host_*.cpp")))
    test = os.path.join(HERE, "selftest_host_collate.cpp")
    exes = {}
    for name, flags in SANITIZERS.items():
        exe = os.path.join(out_dir, f"selftest_host_{name}")
        if _stale(exe, hsrcs + [test]):
            _run(["g++", "-O1", "-g", "-std=c++17", "-pthread"] + flags + ["-o", exe, test] + hsrcs)
        exes[name] = exe
    if verbose:
        print("built", " ".join(exes.values()))
    return exes


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--sanitize", action="store_true",
                    help="also build the host runtime self-test under ASan+UBSan and TSan (build/sanitize/)")
    a = ap.parse_args()
    try:
        build(a.jobs, a.debug, a.clean, verbose=True)
        if a.sanitize:
            build_sanitized(verbose=True)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
