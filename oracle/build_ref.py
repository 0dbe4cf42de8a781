"""Build the REFERENCE Cython kernel module into oracle/_ref/ (test infrastructure only).

Recipe: the reference's own `utils/training_sdg_inner.pyx` + `utils/voidptr.h`
are read from /root/reference (never copied into the repo), cythonized in a scratch directory
with the reference's directives (`cython_utils.py:6-8`: boundscheck/wraparound off, cdivision on)
plus `language_level=2` and `legacy_implicit_noexcept=True` (Cython 3 otherwise inserts
GIL-acquiring error checks after every BLAS call), compiled with -O3, and ONLY the resulting
shared object lands in oracle/_ref/ (git-ignored, and listed in .gpurunignore: it never reaches
the GPU box -- the reference stays in this container).

The module links scipy's bundled BLAS through capsules at import time (pyx:76-86), exactly as the
reference does.  It is used (a) to generate the golden fixtures under tests/golden/ and (b) to
calibrate the CPU restatement that bench.py times as `cpu_baseline` kind "port"
(scripts/calibrate_cpu.py -> profiles/r02_cpu_calibration.json).  Nothing on the product path
imports it.

Usage:  python oracle/build_ref.py   (no-op with a message when /root/reference is absent)
"""
import os
import shutil
import sys
import sysconfig
import subprocess
import tempfile

REF = os.environ.get("COME_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_ref")


def main():
    src = os.path.join(REF, "utils", "training_sdg_inner.pyx")
    if not os.path.isfile(src):
        print("build_ref: %s not present; keeping prebuilt oracle/_ref (if any)" % src)
        return None
    import numpy
    from Cython.Build import cythonize
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="come_ref_")
    try:
        shutil.copy(src, tmp)
        shutil.copy(os.path.join(REF, "utils", "voidptr.h"), tmp)
        pyx = os.path.join(tmp, "training_sdg_inner.pyx")
        cythonize([pyx], quiet=True, compiler_directives={
            "boundscheck": False, "wraparound": False, "cdivision": True,
            "language_level": 2, "legacy_implicit_noexcept": True})
        csrc = os.path.join(tmp, "training_sdg_inner.c")
        ext = sysconfig.get_config_var("EXT_SUFFIX")
        so = os.path.join(OUT, "training_sdg_inner" + ext)
        cmd = ["gcc", "-shared", "-fPIC", "-O3", "-fno-strict-aliasing",
               "-DNPY_NO_DEPRECATED_API=NPY_1_7_API_VERSION",
               "-I" + sysconfig.get_paths()["include"], "-I" + numpy.get_include(), "-I" + tmp,
               csrc, "-o", so]
        subprocess.check_call(cmd)
        print("build_ref: built", so)
        return so
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(0 if main() is not None or not os.path.isdir(REF) else 1)
