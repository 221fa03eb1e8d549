"""In-tree build of the native core (``shellac_amd/_shellac_core*.so``).

HIP translation units (``*.hip``) are compiled by ``hipcc --offload-arch=gfx950``;
host C++ units (``*.cc``) by ``g++`` against the HIP runtime headers; everything
is linked by ``hipcc -shared`` against ``libamdhip64``, ROCTX (timeline markers) and ``libz``. Objects are
cached under ``build/obj`` and rebuilt when the source or any ``csrc`` header is
newer. No JIT cache: the ``.so`` lands in the package directory so it travels
to the GPU box with the repository snapshot.

Usage: ``python -m shellac_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("SHELLAC_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = os.path.join(PKG, "_shellac_core" + EXT)


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _py_include() -> str:
    return sysconfig.get_paths()["include"]


def _headers() -> list[str]:
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]


def _sources() -> list[str]:
    return sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".cc", ".hip"))
    )


def _obj_for(src: str) -> str:
    return os.path.join(OBJ, os.path.basename(src) + ".o")


def _stale(src: str, obj: str, hdr_mtime: float) -> bool:
    if not os.path.exists(obj):
        return True
    om = os.path.getmtime(obj)
    return om < os.path.getmtime(src) or om < hdr_mtime


def _compile_cmd(src: str, obj: str) -> list[str]:
    common = [
        "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
        f"-I{CSRC}", f"-I{_pybind_include()}", f"-I{_py_include()}",
        f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__", "-fvisibility=hidden",
    ]
    if src.endswith(".hip"):
        return [f"{ROCM}/bin/hipcc", "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                *common, "-c", src, "-o", obj]
    return ["g++", *common, "-pthread", "-c", src, "-o", obj]


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    hdr_mtime = max((os.path.getmtime(h) for h in _headers()), default=0.0)
    srcs = _sources()
    todo = [s for s in srcs if force or _stale(s, _obj_for(s), hdr_mtime)]
    jobs = jobs or min(8, os.cpu_count() or 4)

    def run(src: str) -> tuple[str, int, str]:
        cmd = _compile_cmd(src, _obj_for(src))
        p = subprocess.run(cmd, capture_output=True, text=True)
        return src, p.returncode, (p.stdout + p.stderr)

    failed = []
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for src, rc, out in ex.map(run, todo):
                name = os.path.basename(src)
                if rc != 0:
                    failed.append(name)
                    sys.stderr.write(f"[shellac build] FAILED {name}\n{out}\n")
                elif verbose or "warning" in out:
                    sys.stderr.write(f"[shellac build] {name}\n{out}" if out.strip() else "")
    if failed:
        raise RuntimeError(f"shellac_amd native build failed: {', '.join(failed)}")
    objs = [_obj_for(s) for s in srcs]
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(TARGET) or os.path.getmtime(TARGET) < newest:
        cmd = [f"{ROCM}/bin/hipcc", "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs,
               "-o", TARGET + ".tmp", f"-L{ROCM}/lib", "-lamdhip64", "-lrocprofiler-sdk-roctx", "-lz", "-ldl",
               "-lpthread",
               f"-Wl,-rpath,{ROCM}/lib"]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"shellac_amd link failed:\n{p.stdout}{p.stderr}")
        os.replace(TARGET + ".tmp", TARGET)
    return TARGET


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.jobs, verbose=a.verbose))


if __name__ == "__main__":
    main()
