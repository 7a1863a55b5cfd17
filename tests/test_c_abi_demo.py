"""The C ABI used from plain C (tests/c_abi_demo.c): it compiles and links against
libdlagg.so here; on the GPU box it runs and checks itself bit-for-bit."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "decentralized-learning_amd", "lib")


def _build(tmp_path):
    from accdfl_amd import _lib

    _lib.build()
    exe = str(tmp_path / "c_abi_demo")
    cmd = ["gcc", "-std=c11", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tests", "c_abi_demo.c"),
           "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
           "-L" + LIBDIR, "-ldlagg", "-Wl,-rpath," + LIBDIR, "-L/opt/rocm/lib", "-lamdhip64",
           "-Wl,-rpath,/opt/rocm/lib", "-lm", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_c_program_builds_against_the_abi(tmp_path):
    assert os.path.exists(_build(tmp_path))


@pytest.mark.gpu
def test_c_program_runs_bit_exact(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c_abi_demo ok" in r.stdout
