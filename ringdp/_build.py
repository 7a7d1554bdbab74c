"""Build driver for ringdp's native extension (``ringdp/_C*.so``).

Everything is compiled in-tree so the built object travels with the repository snapshot:

* ``csrc/kernels/*.hip``  -> ``hipcc --offload-arch=gfx950 -O3`` (pure HIP, no torch headers:
  kernels take raw pointers + a ``hipStream_t``).
* ``csrc/**/*.cpp``        -> host C++17 against the installed PyTorch-ROCm headers (runtime:
  stores, process groups, reducer, op wrappers, pybind bindings).
* link                     -> one shared object against torch's bundled HIP runtime + RCCL.

Incremental: an object is rebuilt only when its source or any header under ``csrc/`` is newer.

Sanitized host build (SURVEY.md §5 race/sanitizer row): ``--sanitize address`` compiles the host
C++ runtime (stores, host ring, RCCL PG, reducer, bindings) with ``-fsanitize=address`` into
``build/asan/`` (device code unchanged, no GPU sanitizer), linked by g++ against gcc's libasan.
Load it with ``RINGDP_EXT_PATH=<that .so>`` and ``LD_PRELOAD=libasan.so`` (tools/asan_check.sh).
Usage: ``python __graft_entry__.py build`` (the package import needs the built extension, so the
driver is loaded by file path there).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
OUT_DIR = ROOT / "ringdp"
EXT_NAME = "_C"
ARCH = os.environ.get("RINGDP_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_paths():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    lib = tdir / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return OUT_DIR / f"{EXT_NAME}{suffix}"


def _sources():
    hip = sorted(CSRC.rglob("*.hip"))
    cpp = sorted(CSRC.rglob("*.cpp"))
    return hip, cpp


def _headers_mtime() -> float:
    hs = list(CSRC.rglob("*.h")) + list(CSRC.rglob("*.hpp")) + list(CSRC.rglob("*.cuh"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _obj_for(src: Path, build_dir: Path = BUILD) -> Path:
    rel = src.relative_to(CSRC)
    return build_dir / (str(rel).replace(os.sep, "__") + ".o")


def _hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else (shutil.which("hipcc") or "hipcc")


def _cxx() -> str:
    return os.environ.get("RINGDP_CXX", shutil.which("g++") or "c++")


def _compile_cmd(src: Path, obj: Path, sanitize: str | None = None):
    inc, _lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-fPIC", "-std=c++17", f"-I{CSRC}"]
    if src.suffix == ".hip":
        # Device code: pure HIP for CDNA4.  No torch headers here on purpose.
        return [
            _hipcc(), f"--offload-arch={ARCH}", "-O3", "-fno-gpu-rdc", "-munsafe-fp-atomics",
            *common, "-c", str(src), "-o", str(obj),
        ]
    defs = [
        "-D__HIP_PLATFORM_AMD__=1",  # selects the AMD flavour of the HIP runtime headers
        "-DUSE_ROCM=1",               # PyTorch-ROCm header configuration
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
    ]
    incs = [f"-I{p}" for p in inc] + [f"-I{py_inc}", f"-I{ROCM / 'include'}"]
    opt = ["-O2", "-g0"] if not sanitize else ["-O1", "-g", f"-fsanitize={sanitize}", "-fno-omit-frame-pointer"]
    return [_cxx(), *opt, "-Wno-deprecated-declarations", *defs, *common, *incs,
            "-c", str(src), "-o", str(obj)]


def _link_cmd(objs, out: Path):
    _inc, lib, _abi = _torch_paths()
    libs = ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-lamdhip64", "-lrccl"]
    return [
        _hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc", *map(str, objs),
        f"-L{lib}", *libs, f"-Wl,-rpath,{lib}", "-Wl,--no-as-needed", "-o", str(out),
    ]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n  " + " ".join(cmd) + "\n" + r.stdout[-8000:])
    return r.stdout


def _link_cmd_sanitized(objs, out: Path, sanitize: str):
    _inc, lib, _abi = _torch_paths()
    libs = ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-lamdhip64", "-lrccl"]
    return [_cxx(), "-shared", "-fPIC", f"-fsanitize={sanitize}", *map(str, objs), f"-L{lib}",
            f"-L{ROCM / 'lib'}", *libs, f"-Wl,-rpath,{lib}", "-Wl,--no-as-needed", "-o", str(out)]


def build(force: bool = False, jobs: int | None = None, verbose: bool = False,
          sanitize: str | None = None) -> Path:
    """Compile + link the extension; returns the path of the built shared object."""
    bdir = BUILD if not sanitize else ROOT / "build" / f"native-{sanitize}"
    bdir.mkdir(parents=True, exist_ok=True)
    hip, cpp = _sources()
    hdr_t = _headers_mtime()
    todo = []
    objs = []
    for src in hip + cpp:
        # device code is never sanitized: reuse the regular objects
        obj = _obj_for(src, BUILD if (sanitize and src.suffix == ".hip") else bdir)
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_t):
            todo.append((src, obj))
    jobs = jobs or int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 4)))
    if todo:
        if verbose:
            print(f"[ringdp build] compiling {len(todo)} file(s) with {jobs} job(s)", flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_run, _compile_cmd(s, o, sanitize if s.suffix == ".cpp" else None)): s
                    for s, o in todo}
            for f in cf.as_completed(futs):
                f.result()
                if verbose:
                    print(f"  built {futs[f].relative_to(ROOT)}", flush=True)
    out = ext_path() if not sanitize else ROOT / "build" / sanitize / ext_path().name
    out.parent.mkdir(parents=True, exist_ok=True)
    newest = max(o.stat().st_mtime for o in objs)
    if force or todo or not out.exists() or out.stat().st_mtime < newest:
        tmp = out.with_suffix(".tmp.so")
        _run(_link_cmd(objs, tmp) if not sanitize else _link_cmd_sanitized(objs, tmp, sanitize))
        os.replace(tmp, out)
        if verbose:
            print(f"[ringdp build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--sanitize", type=str, default=None, help="host-code sanitizer, e.g. 'address'")
    a = ap.parse_args(argv)
    p = build(force=a.force, jobs=a.jobs, verbose=True, sanitize=a.sanitize)
    print(p)


if __name__ == "__main__":
    sys.exit(main())
