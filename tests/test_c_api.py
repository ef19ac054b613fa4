"""The C ABI as a C program uses it: tests/ctest/rure_ctest.c (the cases of
the reference's regex-capi/ctest/test.c) compiled with gcc against
include/rure_amd.h and linked to librure_amd.so.  Building runs on CPU; the
run needs the GPU (every search launches kernels)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "regex_amd", "lib")


def build(tmp_path):
    exe = str(tmp_path / "rure_ctest")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-o", exe,
                           os.path.join(ROOT, "tests", "ctest", "rure_ctest.c"),
                           "-I", os.path.join(ROOT, "include"), "-L", LIB, "-lrure_amd",
                           "-Wl,-rpath," + LIB, "-Wl,--allow-shlib-undefined"])
    return exe


def test_ctest_builds(tmp_path):
    assert os.path.exists(build(tmp_path))


@pytest.mark.gpu
def test_ctest_runs(tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


def build_batch(tmp_path):
    """tests/ctest/batch_ctest.c: the batched device entry points from C, with
    device buffers from the HIP runtime (C API, hip_runtime_api.h)."""
    exe = str(tmp_path / "batch_ctest")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-o", exe,
                           os.path.join(ROOT, "tests", "ctest", "batch_ctest.c"),
                           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                           "-L", LIB, "-lrure_amd", "-L", "/opt/rocm/lib", "-lamdhip64",
                           "-Wl,-rpath," + LIB, "-Wl,-rpath,/opt/rocm/lib", "-Wl,--allow-shlib-undefined"])
    return exe


def test_batch_ctest_builds(tmp_path):
    assert os.path.exists(build_batch(tmp_path))


@pytest.mark.gpu
def test_batch_ctest_runs(tmp_path):
    exe = build_batch(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout
