"""CPU checks of the C-ABI boundary: the engine library loads, exports every
function include/dmclock_gpu.h declares, and the Python record layouts match
the C structs (checked by compiling a tiny C program against the header)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from dmclock_amd import _abi
from dmclock_amd import gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dmclock_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dmc_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = gpu.lib()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding wires every one of them
    assert set(names) <= set(gpu.EXPORTS), set(names) - set(gpu.EXPORTS)


def test_abi_version_matches_header():
    """DMC_ABI_VERSION (option ids and dmc_counters changed without
    a way to detect it): the library, the header and the binding agree."""
    src = open(HEADER).read()
    v = int(re.search(r"#define DMC_ABI_VERSION (\d+)", src).group(1))
    assert gpu.lib().dmc_abi_version() == v == _abi.ABI_VERSION
    assert "#define DMC_OPT_FAULT 13" in src and _abi.OPT_FAULT == 13


def test_retired_option_and_sized_counters_need_a_queue():
    """option 9 (the retired DMC_OPT_PREDICT) and the size-checked counters
    query reject a null queue without touching a device"""
    L = gpu.lib()
    assert L.dmc_queue_set_option(None, 9, 1) == _abi.DMC_EINVAL
    buf = ctypes.create_string_buffer(64)
    assert L.dmc_queue_counters_sized(None, buf, 64, 0) == _abi.DMC_EINVAL


def test_queue_create_fails_loudly_without_device():
    """No CPU fallback: without a HIP device queue creation returns an error
    (DMC_EDEVICE) and the binding raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(gpu.DmcError):
        gpu.GpuQueue(max_clients=8, ring_capacity=8)


def test_invalid_params_rejected():
    L = gpu.lib()
    p = _abi.QueueParams()
    p.max_clients = 8
    p.ring_capacity = 6  # not a power of two
    h = ctypes.c_void_p()
    assert L.dmc_queue_create(ctypes.byref(p), ctypes.byref(h)) == _abi.DMC_EINVAL
    p.ring_capacity = 8
    p.delayed = 1
    p.at_limit = _abi.AT_LIMIT_REJECT  # Reject needs immediate tags (:856-857)
    assert L.dmc_queue_create(ctypes.byref(p), ctypes.byref(h)) == _abi.DMC_EINVAL


C_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "dmclock_gpu.h"
#define P(T, F) printf(#T "." #F " %zu\n", offsetof(T, F))
int main(void) {
  printf("dmc_request %zu\n", sizeof(dmc_request));
  printf("dmc_decision %zu\n", sizeof(dmc_decision));
  printf("dmc_queue_params %zu\n", sizeof(dmc_queue_params));
  printf("dmc_pull_result %zu\n", sizeof(dmc_pull_result));
  printf("dmc_client_state %zu\n", sizeof(dmc_client_state));
  printf("dmc_stats %zu\n", sizeof(dmc_stats));
  printf("dmc_counters %zu\n", sizeof(dmc_counters));
  printf("dmc_group_tracker %zu\n", sizeof(dmc_group_tracker));
  P(dmc_group_tracker, comp_rho);
  P(dmc_counters, single_steps); P(dmc_counters, max_bin);
  P(dmc_counters, bin_splits);
  P(dmc_request, time); P(dmc_request, delta); P(dmc_request, handle);
  P(dmc_decision, tag_r); P(dmc_decision, slot); P(dmc_decision, flags);
  P(dmc_queue_params, reject_threshold); P(dmc_queue_params, device);
  P(dmc_pull_result, when); P(dmc_pull_result, n_priority);
  return 0;
}
"""


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(C_PROBE)
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"),
                           str(src), "-o", str(exe)])
    out = dict(line.rsplit(" ", 1) for line in
               subprocess.check_output([str(exe)]).decode().splitlines())
    out = {k: int(v) for k, v in out.items()}
    assert out["dmc_request"] == _abi.REQUEST_DTYPE.itemsize
    assert out["dmc_decision"] == _abi.DECISION_DTYPE.itemsize
    assert out["dmc_queue_params"] == ctypes.sizeof(_abi.QueueParams)
    assert out["dmc_pull_result"] == ctypes.sizeof(_abi.PullResult)
    assert out["dmc_client_state"] == ctypes.sizeof(_abi.ClientState)
    assert out["dmc_stats"] == ctypes.sizeof(_abi.Stats)
    assert out["dmc_counters"] == ctypes.sizeof(_abi.Counters)
    assert out["dmc_group_tracker"] == ctypes.sizeof(_abi.GroupTracker)
    assert out["dmc_group_tracker.comp_rho"] == _abi.GroupTracker.comp_rho.offset
    assert out["dmc_counters.single_steps"] == _abi.Counters.single_steps.offset
    assert out["dmc_counters.max_bin"] == _abi.Counters.max_bin.offset
    assert out["dmc_counters.bin_splits"] == _abi.Counters.bin_splits.offset
    assert out["dmc_request.time"] == _abi.REQUEST_DTYPE.fields["time"][1]
    assert out["dmc_request.delta"] == _abi.REQUEST_DTYPE.fields["delta"][1]
    assert out["dmc_request.handle"] == _abi.REQUEST_DTYPE.fields["handle"][1]
    assert out["dmc_decision.tag_r"] == _abi.DECISION_DTYPE.fields["tag_r"][1]
    assert out["dmc_decision.slot"] == _abi.DECISION_DTYPE.fields["slot"][1]
    assert out["dmc_decision.flags"] == _abi.DECISION_DTYPE.fields["flags"][1]
    assert out["dmc_queue_params.reject_threshold"] == \
        _abi.QueueParams.reject_threshold.offset
    assert out["dmc_queue_params.device"] == _abi.QueueParams.device.offset
    assert out["dmc_pull_result.when"] == _abi.PullResult.when.offset
    assert out["dmc_pull_result.n_priority"] == _abi.PullResult.n_priority.offset


def test_make_requests_broadcast():
    r = _abi.make_requests([1, 2, 3], 5.0, costs=2)
    assert r["cost"].tolist() == [2, 2, 2]
    assert r["time"].tolist() == [5.0] * 3
    assert r["handle"].tolist() == [0, 1, 2]
    assert np.all(r["delta"] == 1)
