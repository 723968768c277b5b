"""Build script for accelerate_hpc_test_amd and its in-tree MI355X (gfx950) extension.

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

produces `accelerate_hpc_test_amd/_C.*.so` next to the Python sources (the in-tree .so is what the GPU box
loads). `__graft_entry__.build()` runs the same thing.
"""

import glob
import os
import re

from setuptools import find_packages, setup

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")


def _touch_if_includes_changed(sources, include_dirs):
    """The ninja build recompiles a .hip source only when that file changes, not when a file it #includes does (no
    depfiles for hipcc here): the csrc/debug shims are one-line includes of the kernel sources, and every kernel
    includes kernels/common.h. Give each source the newest mtime of its quoted-include closure so ninja sees it."""
    pat = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)

    def closure(path, seen):
        if path in seen or not os.path.isfile(path):
            return
        seen.add(path)
        with open(path, encoding="utf-8", errors="replace") as f:
            text = f.read()
        for inc in pat.findall(text):
            for d in [os.path.dirname(path)] + list(include_dirs):
                cand = os.path.normpath(os.path.join(d, inc))
                if os.path.isfile(cand):
                    closure(cand, seen)
                    break

    for src in sources:
        deps = set()
        closure(src, deps)
        newest = max(os.path.getmtime(p) for p in deps)
        if newest > os.path.getmtime(src):
            os.utime(src, (newest, newest))


ext_modules = []
cmdclass = {}
if os.environ.get("ACCELERATE_SKIP_NATIVE_BUILD", "0") != "1":
    from torch.utils.cpp_extension import BuildExtension, CUDAExtension

    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "accelerate_hpc_test_amd", "csrc")
    sources = (
        [os.path.join(root, "bindings.cpp")]
        + sorted(g for g in glob.glob(os.path.join(root, "kernels", "*.hip")) if not g.endswith("_hip.hip"))
        + sorted(glob.glob(os.path.join(root, "runtime", "*.cpp")))
    )
    _touch_if_includes_changed(sources, [os.path.join(root, "kernels")])
    sources = [os.path.relpath(s, os.path.dirname(os.path.abspath(__file__))) for s in sources]
    ext_modules.append(
        CUDAExtension(
            name="accelerate_hpc_test_amd._C",
            sources=sources,
            include_dirs=[os.path.join(root, "kernels")],
            libraries=["hipblaslt"],
            extra_link_args=["-fopenmp"],
            # -fno-slp-vectorize: hipcc's SLP pass pairs scalar f32 multiplies / adds into v_pk_*_f32, which beside MFMAs
            # cost more issue cycles than the two single ops they replace and need v_mov pairs to align their
            # operands (the attention kernels' softmax; MI355X_MICROARCH cycle constants). Explicit vector types
            # still lower to packed ops where the kernels ask for them.
            extra_compile_args={
                "cxx": ["-O3", "-std=c++17", "-fopenmp"],
                "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-fno-slp-vectorize"],
            },
        )
    )
    # Debug build: the same kernels with the device bounds checks compiled in (csrc/debug/* include the
    # real sources under -DACC_DEBUG_BOUNDS), loaded instead of `_C` when ACCELERATE_DEBUG_KERNELS=1.
    # ACCELERATE_BUILD_DEBUG_KERNELS=0 skips it.
    if os.environ.get("ACCELERATE_BUILD_DEBUG_KERNELS", "1") != "0":
        dbg = sorted(glob.glob(os.path.join(root, "debug", "*.hip"))) + sorted(glob.glob(os.path.join(root, "debug", "*.cpp")))
        _touch_if_includes_changed(dbg, [os.path.join(root, "kernels")])
        ext_modules.append(
            CUDAExtension(
                name="accelerate_hpc_test_amd._C_debug",
                sources=[os.path.relpath(s, os.path.dirname(os.path.abspath(__file__))) for s in dbg],
                include_dirs=[os.path.join(root, "kernels")],
                libraries=["hipblaslt"],
                extra_link_args=["-fopenmp"],
                extra_compile_args={
                    "cxx": ["-O3", "-std=c++17", "-fopenmp", "-DACC_DEBUG_BOUNDS"],
                    "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-fno-slp-vectorize", "-DACC_DEBUG_BOUNDS"],
                },
            )
        )
    cmdclass = {"build_ext": BuildExtension.with_options(use_ninja=True)}

console_scripts = [
    "accelerate-amd=accelerate_hpc_test_amd.commands.accelerate_cli:main",
    "accelerate-amd-launch=accelerate_hpc_test_amd.commands.launch:main",
    "accelerate-amd-config=accelerate_hpc_test_amd.commands.config:main",
    "accelerate-amd-estimate-memory=accelerate_hpc_test_amd.commands.estimate:main",
    "accelerate-amd-merge-weights=accelerate_hpc_test_amd.commands.merge:main",
]
# Opt-in drop-in names of the reference (setup.py:70-78); off by default so an installed upstream `accelerate` is not
# shadowed. Also available after installation: `accelerate-amd aliases install`.
if os.environ.get("ACCELERATE_AMD_INSTALL_ALIASES", "0") == "1":
    console_scripts += [
        "accelerate=accelerate_hpc_test_amd.commands.accelerate_cli:main",
        "accelerate-launch=accelerate_hpc_test_amd.commands.launch:main",
        "accelerate-config=accelerate_hpc_test_amd.commands.config:main",
        "accelerate-estimate-memory=accelerate_hpc_test_amd.commands.estimate:main",
        "accelerate-merge-weights=accelerate_hpc_test_amd.commands.merge:main",
    ]

setup(
    name="accelerate_hpc_test_amd",
    version="0.1.0",
    description="MI355X-native training-loop framework with the Accelerate API (RCCL/xGMI, HIP/CDNA4 kernels)",
    packages=find_packages(include=["accelerate_hpc_test_amd", "accelerate_hpc_test_amd.*"]),
    python_requires=">=3.10",
    entry_points={"console_scripts": console_scripts},
    ext_modules=ext_modules,
    cmdclass=cmdclass,
)
