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


def test_facade_client_id_types(tmp_path):
    """the facade instantiates for client ids with and without std::hash
    (the per-call lookup uses a hash index only when C is hashable; the
    reference needs only operator<)"""
    src = tmp_path / "ids.cc"
    src.write_text(
        '#include "dmclock_server.h"\n'
        "struct NoHashClient {\n"
        "  int v;\n"
        "  bool operator<(const NoHashClient& o) const { return v < o.v; }\n"
        "};\n"
        "struct Req { int x; };\n"
        "template class crimson::dmclock::PullPriorityQueue<NoHashClient, Req>;\n"
        "template class crimson::dmclock::PushPriorityQueue<NoHashClient, Req>;\n"
        "template class crimson::dmclock::PullPriorityQueue<int, Req>;\n"
        "static_assert(!crimson::dmclock::detail::has_std_hash<NoHashClient>::value);\n"
        "static_assert(crimson::dmclock::detail::has_std_hash<int>::value);\n")
    root = os.path.dirname(HERE)
    out = subprocess.run(["g++", "-std=c++17", "-fsyntax-only",
                          "-I", os.path.join(root, "dmclock_amd", "include"),
                          "-I", os.path.join(root, "include"), str(src)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
