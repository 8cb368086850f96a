"""`ds_report`: native-op build/compat table and environment summary (reference `env_report.py:30-194`)."""
import argparse
import os
import shutil
import subprocess

import torch

GREEN, RED, YELLOW, END = "\033[92m", "\033[91m", "\033[93m", "\033[0m"
OKAY, WARNING, FAIL = f"{GREEN}[OKAY]{END}", f"{YELLOW}[WARNING]{END}", f"{RED}[FAIL]{END}"
INFO = "[INFO]"


def op_report(verbose=True):
    from .ops import op_builder
    print("-" * 80)
    print("DeepSpeed (MI355X) native op report")
    print("-" * 80)
    print("Every extension is AOT-compiled in-tree for gfx950 (ops/lib/*.so); 'built' means the .so is present,\n"
          "'compatible' means the toolchain to (re)build it exists here.")
    print("-" * 80)
    print(f"{'op name':<24}{'extension':<14}{'built':<16}{'compatible':<16}")
    print("-" * 80)
    for name, b in sorted(op_builder.ALL_OPS.items()):
        ext = b.EXT or "(python)"  # builders without native code have nothing to build
        built = OKAY if b.EXT is None or op_builder.is_built(b.EXT) else f"{YELLOW}[NO]{END}"
        compat = OKAY if b().is_compatible() else FAIL
        print(f"{name:<24}{ext:<14}{built:<25}{compat}")
    print("-" * 80)


def _cmd(args):
    try:
        return subprocess.run(args, capture_output=True, text=True, timeout=20).stdout.strip()
    except Exception:
        return ""


def ninja_installed():
    try:
        import ninja  # noqa: F401
        return True
    except ImportError:
        return shutil.which("ninja") is not None


def hipcc_version():
    """Version line of the HIP compiler, or None when hipcc is not installed."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        return None
    lines = _cmd([hipcc, "--version"]).splitlines()
    return lines[0] if lines else None


nvcc_version = hipcc_version  # the reference's name for "device compiler version"


def human_readable_size(size):
    units = ["B", "KB", "MB", "GB", "TB"]
    i = 0
    size = float(size)
    while size >= 1024 and i < len(units) - 1:
        size /= 1024
        i += 1
    return f"{size:.2f} {units[i]}"


def get_shm_size():
    """(human-readable size of /dev/shm, warning or None): RCCL and the host shm all-reduce need room there."""
    try:
        st = os.statvfs("/dev/shm")
    except OSError as e:
        return "UNKNOWN", str(e)
    size = st.f_frsize * st.f_blocks
    warn = None
    if size < 512 * 1024**2:
        warn = (f"/dev/shm is {human_readable_size(size)}: multi-process collectives may fail; under docker pass "
                f"--shm-size=1g or larger")
    return human_readable_size(size), warn


def parse_arguments():
    import argparse
    parser = argparse.ArgumentParser()
    parser.add_argument("--hide_operator_status", action="store_true",
                        help="Suppress display of installation and compatibility statuses of DeepSpeed operators.")
    parser.add_argument("--hide_errors_and_warnings", action="store_true", help="Suppress warning and error messages.")
    return parser.parse_args()


def debug_report():
    from . import __version__
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    ver = ""
    for f in (os.path.join(rocm, ".info", "version"), os.path.join(rocm, ".info", "version-dev")):
        if os.path.exists(f):
            ver = open(f).read().strip()
            break
    rows = [
        ("torch install path", os.path.dirname(torch.__file__)),
        ("torch version", torch.__version__),
        ("torch HIP version", getattr(torch.version, "hip", None)),
        ("ROCm path / version", f"{rocm} {ver}"),
        ("hipcc", _cmd([hipcc, "--version"]).splitlines()[0] if os.path.exists(hipcc) else "not found"),
        ("deepspeedsyclsupport_amd install path", os.path.dirname(os.path.abspath(__file__))),
        ("deepspeedsyclsupport_amd version", __version__),
        ("target arch", os.environ.get("DS_ROCM_ARCH", os.environ.get("PYTORCH_ROCM_ARCH", "gfx950"))),
        ("GPU available", torch.cuda.is_available()),
        ("ninja", ninja_installed()),
        ("shared memory (/dev/shm) size", get_shm_size()[0]),
    ]
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        rows += [("GPU 0", f"{p.name} ({getattr(p, 'gcnArchName', '?')}), {p.total_memory / 2**30:.0f} GiB, "
                  f"{p.multi_processor_count} CUs"), ("device count", torch.cuda.device_count())]
    rows.append(("distributed backends", ", ".join(b for b in ("nccl", "gloo", "mpi")
                                                     if getattr(torch.distributed, f"is_{b}_available")())))
    print("DeepSpeed general environment info:")
    for k, v in rows:
        print(f"{k} {'.' * (40 - len(k))} {v}")


def main(hide_operator_status=False, hide_errors_and_warnings=False):
    if not hide_operator_status:
        op_report(verbose=not hide_errors_and_warnings)
    debug_report()


def cli_main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hide_operator_status", action="store_true")
    ap.add_argument("--hide_errors_and_warnings", action="store_true")
    a = ap.parse_args()
    main(a.hide_operator_status, a.hide_errors_and_warnings)


if __name__ == "__main__":
    cli_main()
