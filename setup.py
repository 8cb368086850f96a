"""Packaging of the MI355X-native framework (reference `setup.py`).

    pip install .                 # Python package + launcher scripts; native ops are built in-tree on first use
    DS_BUILD_OPS=1 pip install .  # pre-build every gfx950 / host extension (hipcc + g++ through ninja) first

There is a single target: ROCm / gfx950. `DS_BUILD_<OP>=0/1` switches of the reference that pick individual ops are
accepted and ignored with a note: the extensions here are two shared objects (device ops, host ops), not one per op.
"""
import os
import sys

from setuptools import find_packages, setup

ROOT = os.path.dirname(os.path.abspath(__file__))


def version():
    ns = {}
    with open(os.path.join(ROOT, "deepspeedsyclsupport_amd", "__init__.py")) as f:
        for line in f:
            if line.startswith("__version__"):
                exec(line, ns)
                break
    return ns.get("__version__", "0.0.0")


def prebuild():
    os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    sys.path.insert(0, ROOT)
    import __graft_entry__ as entry
    entry.build()


if os.environ.get("DS_BUILD_OPS", "0") == "1":
    prebuild()
for key in [k for k in os.environ if k.startswith("DS_BUILD_") and k != "DS_BUILD_OPS"]:
    print(f"[setup] {key} is ignored: the native ops build as two shared objects (see ops/op_builder.py)")

setup(
    name="deepspeedsyclsupport_amd",
    version=version(),
    description="MI355X-native ZeRO training and inference framework (PyTorch-ROCm, HIP/CDNA4 kernels, RCCL)",
    packages=find_packages(include=["deepspeedsyclsupport_amd", "deepspeedsyclsupport_amd.*"]),
    package_data={"deepspeedsyclsupport_amd": ["ops/csrc/**/*", "ops/lib/*.so"]},
    include_package_data=True,
    scripts=[os.path.join("bin", s) for s in ("deepspeed", "deepspeed.pt", "ds", "ds_report", "ds_ssh", "ds_bench",
                                              "ds_elastic", "dsr")],
    python_requires=">=3.8",
    install_requires=["torch", "numpy", "pydantic>=2", "psutil", "packaging", "tqdm", "ninja"],
    extras_require={"inf": ["transformers", "safetensors"], "sparse_attn": [], "autotuning": ["tabulate"]},
    classifiers=["Programming Language :: Python :: 3", "Operating System :: POSIX :: Linux"],
)
