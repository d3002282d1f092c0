"""In-tree build of the apneauq HIP extension for gfx950 (MI355X).

Every ``*.hip`` file under ``csrc/`` is compiled by ``hipcc --offload-arch=gfx950`` and the
torch.library bindings (``bindings.cpp``) by the host C++ compiler; the result is linked into
``<package>/_apneauq_hip.so`` and loaded with ``torch.ops.load_library``.  No hipify step, no
JIT cache: the ``.so`` sits in the source tree so it travels with the repository snapshot.

Usage: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.csrc.build [--force] [-j N]``

Debug variants (SURVEY §5 "Race detection / sanitizers"):

* ``APNEAUQ_DEBUG=1``: kernels are built with ``-DAPNEAUQ_DEBUG`` — device ``assert``s on every
  launch-geometry / index invariant the kernels rely on (grid vs. item count, member / window /
  row bounds) — and the host side with ``-g -fno-omit-frame-pointer``.  Run with
  ``AMD_SERIALIZE_KERNEL=3`` to attribute a failing assert to its launch.
* ``APNEAUQ_HOST_SANITIZE=address,undefined``: ``-fsanitize=`` on the host objects only (GPU
  sanitizers are unavailable on the pool); load with ``LD_PRELOAD=$(gcc -print-file-name=libasan.so)``.

Both flags are part of the build stamp, so switching variants rebuilds.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
SO_NAME = "_apneauq_hip.so"
SO_PATH = os.environ.get("APNEAUQ_SO_OUT") or os.path.join(PKG, SO_NAME)  # probe variants: another path
BUILD_DIR = os.path.join(HERE, "build" + ("_" + hashlib.sha1(os.environ.get("APNEAUQ_SO_OUT", "").encode()).hexdigest()[:8] if os.environ.get("APNEAUQ_SO_OUT") else ""))
ARCH = os.environ.get("APNEAUQ_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
DEBUG = os.environ.get("APNEAUQ_DEBUG", "0") not in ("", "0")
HOST_SAN = os.environ.get("APNEAUQ_HOST_SANITIZE", "")
# A/B builds of the x3 layer kernels swap the complete layer table (csrc/x3_layers.hip): every table is
# a correct configuration, only the speed differs (tools/probes/x3_tables/)
X3_TABLE = os.environ.get("APNEAUQ_X3_TABLE", "")
EXTRA = [f'-DAPNEAUQ_X3_TABLE="{os.path.abspath(X3_TABLE)}"'] if X3_TABLE else []
# ... and of the training wgrad kernels (csrc/train_conv.hip WgCfg)
WG_TABLE = os.environ.get("APNEAUQ_WG_TABLE", "")
EXTRA += [f'-DAPNEAUQ_WG_TABLE="{os.path.abspath(WG_TABLE)}"'] if WG_TABLE else []


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    return ce.include_paths(), ce.library_paths()[0], int(torch._C._GLIBCXX_USE_CXX11_ABI)


def sources():
    hip = sorted(os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith(".hip"))
    cpp = sorted(os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith(".cpp"))
    hdr = sorted(os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith(".h"))
    return hip, cpp, hdr


def _hipcc():
    p = os.path.join(ROCM, "bin", "hipcc")
    return p if os.path.exists(p) else shutil.which("hipcc")


def commands():
    incs, libdir, abi = _torch_paths()
    hip, cpp, _ = sources()
    common = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1", "-fPIC", "-O3",
              "-std=c++17", f"-I{HERE}", f"-I{ROCM}/include"]
    if DEBUG:
        common += ["-DAPNEAUQ_DEBUG=1", "-g", "-fno-omit-frame-pointer"]
    host_san = [f"-fsanitize={HOST_SAN}"] if HOST_SAN else []
    cmds = []
    objs = []
    for src in hip:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        san = (["-Xarch_host"] + host_san) if host_san else []
        cmds.append([_hipcc(), f"--offload-arch={ARCH}", "-c", src, "-o", obj, "-ffp-contract=fast",
                     "-munsafe-fp-atomics"] + san + common + EXTRA)
        objs.append(obj)
    py_inc = sysconfig.get_paths()["include"]
    for src in cpp:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        cmds.append(["g++", "-c", src, "-o", obj, f"-I{py_inc}"] + [f"-I{i}" for i in incs] + host_san + common)
        objs.append(obj)
    link = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", SO_PATH + ".tmp"] + objs + [
        f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{libdir}",
        f"-L{ROCM}/lib", "-lamdhip64"] + host_san
    return cmds, link


def _stamp():
    hip, cpp, hdr = sources()
    h = hashlib.sha256()
    for f in hip + cpp + hdr + [os.path.abspath(__file__)]:
        h.update(f.encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(ARCH.encode())
    h.update(f"debug={DEBUG};san={HOST_SAN};extra={EXTRA}".encode())
    return h.hexdigest()


def up_to_date() -> bool:
    stamp_file = SO_PATH + ".stamp"
    if not (os.path.exists(SO_PATH) and os.path.exists(stamp_file)):
        return False
    with open(stamp_file) as f:
        return f.read().strip() == _stamp()


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> str:
    if not force and up_to_date():
        return SO_PATH
    os.makedirs(BUILD_DIR, exist_ok=True)
    cmds, link = commands()
    jobs = jobs or min(8, len(cmds))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with cf.ThreadPoolExecutor(jobs) as ex:
        for warn in ex.map(run, cmds):
            if verbose and warn:
                print(warn)
    run(link)
    os.replace(SO_PATH + ".tmp", SO_PATH)
    with open(SO_PATH + ".stamp", "w") as f:
        f.write(_stamp())
    return SO_PATH


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.force, a.jobs, a.verbose))


if __name__ == "__main__":
    sys.exit(main())
