"""Runs the C++ facade test (tests/cpp/test_facade.cc): the reference's KATs
written against the drop-in crimson::dmclock API of
dmclock_amd/include/dmclock_server.h.  On CPU only the host-side tracker
tests run; with a GPU, every server KAT runs through the engine, with the
facade's default serve kernel (DMC_OPT_SERVE) and with it off."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")
EXE = os.path.join(CPP, "test_facade")


def _build():
    subprocess.check_call(["make", "-s", "-C", CPP])
    return EXE


def test_facade_host_only():
    out = subprocess.run([_build(), "--host-only"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout


@pytest.mark.gpu
def test_facade_gpu():
    out = subprocess.run([_build()], capture_output=True, text=True,
                         timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout


@pytest.mark.gpu
def test_facade_gpu_kernels():
    """the same KATs with the facade's serve kernel off (DMCLOCK_GPU_SERVE=0:
    every single call launches the single-op kernels)"""
    env = dict(os.environ, DMCLOCK_GPU_SERVE="0")
    out = subprocess.run([_build()], capture_output=True, text=True, timeout=300, env=env)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout
