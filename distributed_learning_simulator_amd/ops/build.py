"""Build the in-tree gfx950 extension `_dls_hip` with hipcc (no torch headers needed).

    python -m distributed_learning_simulator_amd.ops.build [--force] [-j N]

Each `csrc/*.hip` is compiled to an object (incremental, by mtime), `csrc/bindings.cpp`
(pybind11) likewise, and everything is linked — with a generated unit holding the sources'
content hash (`source_hash()`, checked at import by ops/hip.py) — into
`distributed_learning_simulator_amd/_dls_hip<EXT_SUFFIX>` — in-tree so it travels with the
repo snapshot to the GPU box. The .so links libamdhip64.so.7 by SONAME; importing torch first
makes it bind to torch's bundled HIP runtime (one runtime per process).
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "distributed_learning_simulator_amd")
BUILD = os.path.join(ROOT, "build", "hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DLS_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = os.path.join(PKG, "_dls_hip" + EXT_SUFFIX)

COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-mcode-object-version=5",
                "-ffp-contract=fast", "-Wno-unused-result"]
# per-file overrides. compress.hip: the payload decoders must round lo + q·scale twice, like
# the CPU oracle. Under -ffp-contract=fast the backend fuses every fmul+fadd into an FMA,
# whatever the source pragmas say; "on" fuses only within one expression.
FILE_FLAGS = {"compress.hip": ["-ffp-contract=on"]}


def _headers() -> list[str]:
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]


def _unit_hash(src: str, extra: list[str]) -> str:
    """Content hash of one translation unit's inputs: its source, every csrc/ header, the flags."""
    h = hashlib.sha256()
    for d in [src] + sorted(_headers()):
        h.update(d.encode() + b"\0")
        with open(d, "rb") as fh:
            h.update(fh.read())
    h.update(repr((COMMON_FLAGS, extra, ARCH)).encode())
    return h.hexdigest()[:20]


def _needs(obj: str, src: str, extra: list[str] | None = None) -> bool:
    """An object is reused only if its sidecar records the CONTENT hash of the inputs it was
    compiled from (mtimes are not trusted: an edit during a concurrent build, or a checkout,
    can leave an object newer than a source it was not compiled from)."""
    if not os.path.exists(obj):
        return True
    if extra is None:  # (host-check build: mtime rule)
        t = os.path.getmtime(obj)
        return any(os.path.getmtime(d) > t for d in [src] + _headers())
    try:
        with open(obj + ".srchash") as fh:
            return fh.read().strip() != _unit_hash(src, extra)
    except OSError:
        return True


def _compile(src: str, obj: str, extra: list[str], record: bool = False) -> tuple[str, str]:
    """Compile to a temporary object, then move it in place; with `record`, the inputs' content
    hash (taken before and after the compile, which must agree) goes to the sidecar."""
    while True:
        before = _unit_hash(src, extra) if record else ""
        tmp = f"{obj}.{os.getpid()}.tmp.o"
        cmd = [HIPCC, *COMMON_FLAGS, *extra, "-c", src, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if record and _unit_hash(src, extra) != before:
            os.remove(tmp)  # an input changed while compiling: compile again
            continue
        os.replace(tmp, obj)
        if record:
            with open(obj + ".srchash", "w") as fh:
                fh.write(before + "\n")
        return src, r.stderr


STAMP = TARGET + ".srchash"  # content hash of the sources the in-tree .so was linked from


def source_hash() -> str:
    """Content hash of everything that determines the binary: every csrc/ file (name + bytes),
    the compiler flags and the target arch. Compiled INTO the extension (`_C.src_hash()`) and
    checked at import (ops/hip.py), so a binary built from other sources never runs silently."""
    h = hashlib.sha256()
    for f in sorted(os.listdir(CSRC)):
        h.update(f.encode() + b"\0")
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(repr((COMMON_FLAGS, sorted(FILE_FLAGS.items()), ARCH)).encode())
    return h.hexdigest()[:20]


def is_current() -> bool:
    """The in-tree extension exists and was linked from the current sources (its stamp)."""
    try:
        with open(STAMP) as fh:
            return os.path.exists(TARGET) and fh.read().strip() == source_hash()
    except OSError:
        return False


def wait_current(timeout: float = 1800.0) -> None:
    """Block until is_current() (another rank is building), or raise after `timeout` s."""
    t0 = time.time()
    while not is_current():
        if time.time() - t0 > timeout:
            raise TimeoutError(f"extension not rebuilt from the current sources within {timeout:.0f} s")
        time.sleep(1.0)


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> str:
    if not force and is_current():
        return TARGET  # up to date (object files need not be present, e.g. on a GPU box snapshot)
    os.makedirs(BUILD, exist_ok=True)
    import fcntl

    # one build at a time per tree (concurrent builders — a test, a second shell — serialise;
    # the one that waited finds the tree current and returns)
    with open(os.path.join(BUILD, ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and is_current():
            return TARGET
        return _build_locked(force, jobs, verbose)


def _build_locked(force: bool, jobs: int, verbose: bool) -> str:
    import pybind11

    digest = source_hash()
    py_inc = sysconfig.get_paths()["include"]
    units = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hip") or f.endswith(".cpp"):
            src = os.path.join(CSRC, f)
            obj = os.path.join(BUILD, f + ".o")
            extra = [f"-I{CSRC}", *FILE_FLAGS.get(f, [])]
            if f.endswith(".cpp"):
                extra += [f"-I{pybind11.get_include()}", f"-I{py_inc}", "-x", "hip"]
            units.append((src, obj, extra))
    todo = [u for u in units if force or _needs(u[1], u[0], u[2])]
    jobs = jobs or min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8) or 1
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for src, err in ex.map(lambda u: _compile(*u, record=True), todo):
                if verbose:
                    print("compiled", os.path.basename(src), file=sys.stderr)
                if err.strip() and verbose:
                    print(err, file=sys.stderr)
    # the source hash as a one-line translation unit linked into the extension
    hsrc = os.path.join(BUILD, "srchash.cpp")
    with open(hsrc, "w") as fh:
        fh.write(f'extern "C" const char* dls_src_hash() {{ return "{digest}"; }}\n')
    hobj = os.path.join(BUILD, "srchash.o")
    r = subprocess.run(["g++", "-O2", "-fPIC", "-c", hsrc, "-o", hobj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"srchash compile failed: {r.stderr}")
    objs = [u[1] for u in units] + [hobj]
    tmp = TARGET + ".tmp"
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    # a host function left undefined (e.g. declared in dls.h but defined inside an anonymous
    # namespace) links fine into a shared object and only fails at import: dlopen it (RTLD_NOW) in
    # a child process here, on the build machine, instead
    r = subprocess.run([sys.executable, "-c", "import ctypes, sys; ctypes.CDLL(sys.argv[1])", tmp],
                       capture_output=True, text=True)
    if r.returncode != 0:
        os.remove(tmp)
        raise RuntimeError(f"the linked extension does not load:\n{r.stderr.strip()[-2000:]}")
    os.replace(tmp, TARGET)
    if source_hash() != digest:  # a source changed during the build: rebuild what it touched
        return _build_locked(False, jobs, verbose)
    with open(STAMP + ".tmp", "w") as fh:
        fh.write(digest + "\n")
    os.replace(STAMP + ".tmp", STAMP)  # (written last: waiters see it only after the .so is in place)
    return TARGET


SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
             "-fno-omit-frame-pointer", "-g"]
HOST_CHECK = os.path.join(ROOT, "build", "host_asan", "host_check")


def build_host_check(jobs: int = 0) -> str:
    """tests/native/host_check.cpp + every csrc/*.hip with host-side ASan/UBSan:
    the host launch-planning code under sanitizers. Device code is compiled as usual (GPU
    sanitizers are not used). Incremental like `build`."""
    out_dir = os.path.dirname(HOST_CHECK)
    os.makedirs(out_dir, exist_ok=True)
    units = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hip"):
            units.append((os.path.join(CSRC, f), os.path.join(out_dir, f + ".o"),
                          [f"-I{CSRC}", *FILE_FLAGS.get(f, []), *SAN_FLAGS]))
    main_src = os.path.join(ROOT, "tests", "native", "host_check.cpp")
    units.append((main_src, os.path.join(out_dir, "host_check.o"), [f"-I{CSRC}", "-x", "hip", *SAN_FLAGS]))
    todo = [u for u in units if _needs(u[1], u[0])]
    jobs = jobs or min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8) or 1
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda u: _compile(*u), todo))
    objs = [u[1] for u in units]
    if todo or not os.path.exists(HOST_CHECK) or any(os.path.getmtime(o) > os.path.getmtime(HOST_CHECK) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-fsanitize=address,undefined", "-o", HOST_CHECK, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return HOST_CHECK


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=0)
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.j, verbose=True))


if __name__ == "__main__":
    main()
