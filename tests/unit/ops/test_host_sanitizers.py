"""Host sanitizers over the native CPU ops (SURVEY §5.2 [design]): the ds_cpu_ops translation units (CPU Adam /
Adagrad / Lion, async tensor I/O thread pool, POSIX-shm all-reduce) are compiled into a standalone harness
(`tools/sanitize/host_ops_sanitize.cpp`) with AddressSanitizer + UndefinedBehaviorSanitizer; the threaded parts
(I/O pool, shm barrier) run with several I/O requests in flight; any report fails the test. Host code only —
device code cannot be sanitized on this pool. (ThreadSanitizer is not usable here: a TSan build of the harness
segfaults at start-up against the uninstrumented libtorch, so data-race coverage stays with ASan's use-after-free /
overflow checks of the thread pool.)"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
SRC = os.path.join(ROOT, "tools", "sanitize", "host_ops_sanitize.cpp")


def _flags():
    import sysconfig

    import torch
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths()
    libs = ce.library_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    pyinc = sysconfig.get_paths()["include"]
    pylib = sysconfig.get_config_var("LIBDIR")
    pyver = f"python{sys.version_info.major}.{sys.version_info.minor}"
    cflags = ["-std=c++17", "-O1", "-g", "-fopenmp", "-fno-omit-frame-pointer", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations"]
    cflags += [f"-isystem{p}" for p in inc] + [f"-isystem{pyinc}"]
    lflags = [f"-L{p}" for p in libs] + [f"-Wl,-rpath,{p}" for p in libs]
    lflags += [f"-L{pylib}", f"-Wl,-rpath,{pylib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
               f"-l{pyver}", "-lrt", "-lpthread"]
    return cflags, lflags


def _build_and_run(tmp_path, san, parts, extra_c=()):
    """Build the harness with `-fsanitize=san` (sanitizer runtime linked statically into the executable) and run
    each part in its own process: the shm part forks, and GNU OpenMP is not fork-safe once a process has used it."""
    if shutil.which("g++") is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / f"host_ops_{san.replace(',', '_')}")
    cflags, lflags = _flags()
    static = [{"address": "-static-libasan", "undefined": "-static-libubsan"}[x] for x in san.split(",")]
    cmd = ["g++", *cflags, *extra_c, f"-fsanitize={san}", *static, SRC, "-o", exe, *lflags]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ)
    env.update(ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0", OMP_NUM_THREADS="4")
    outs = []
    for what in parts:
        r = subprocess.run([exe, what, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
        out = r.stdout + r.stderr
        assert r.returncode == 0 and "all ok" in r.stdout, f"{san} {what}: " + out[-6000:]
        assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out and \
            "WARNING: ThreadSanitizer" not in out, out[-6000:]
        outs.append(r.stdout)
    return "".join(outs)


def test_host_ops_asan_ubsan(tmp_path):
    out = _build_and_run(tmp_path, "address,undefined", ["optim", "aio", "shm"],
                         ("-fno-sanitize-recover=undefined", ))
    assert "optim ok" in out and "aio ok" in out and "shm ok" in out

