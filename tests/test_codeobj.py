"""The shipped library's gfx950 code object (CPU: reads the .so, runs nothing).

Every kernel of dmclock_amd/libdmclock_gpu.so -- ours, and the scans and
sort of dmc_sort.h that replaced the library ones -- must use no scratch
memory (private segment 0, no dynamic stack): scratch is allocated per
hardware queue by the runtime, and config 5 drives eight queues on eight
hardware queues at once (round 2's open fault sat in the only kernels that
used it, the library radix sort's).  Also checks the code object targets
gfx950.
"""
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("DMC_LIB") or os.path.join(ROOT, "dmclock_amd", "libdmclock_gpu.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def _section(data, name):
    """(offset, size) of an ELF64 section by name"""
    shoff = struct.unpack_from("<Q", data, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    stro = sh(shstrndx)[4]
    for i in range(shnum):
        h = sh(i)
        end = data.index(b"\0", stro + h[0])
        if data[stro + h[0]:end].decode() == name:
            return h[4], h[5]
    raise KeyError(name)


def code_objects(path):
    """the device code objects of the .hip_fatbin offload bundle(s)"""
    data = open(path, "rb").read()
    off, size = _section(data, ".hip_fatbin")
    fb = data[off:off + size]
    out = {}
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = 0
    while True:
        pos = fb.find(magic, pos)
        if pos < 0:
            break
        n = struct.unpack_from("<Q", fb, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "amdgcn" in triple:
                out[triple] = fb[pos + eo:pos + eo + es]
        pos = p
    return out


@pytest.fixture(scope="module")
def notes(tmp_path_factory):
    if not os.path.exists(LIB):
        pytest.skip("engine library not built")
    cos = code_objects(LIB)
    assert cos, "no amdgcn code object in the library"
    assert all("gfx950" in t for t in cos), list(cos)
    out = {}
    for i, (t, co) in enumerate(cos.items()):
        f = tmp_path_factory.mktemp("co") / f"co{i}.elf"
        f.write_bytes(co)
        out[t] = subprocess.check_output([READELF, "--notes", str(f)]).decode()
    return out


def kernels(text):
    """(name, private segment bytes, dynamic stack) per kernel"""
    blocks = re.split(r"\n\s+- \.", text)
    res = []
    for b in blocks:
        m = re.search(r"\.name:\s+(\S+)", b)
        p = re.search(r"\.private_segment_fixed_size:\s+(\d+)", b)
        if not m or not p or not re.search(r"\.kernarg_segment_size", b):
            continue
        d = re.search(r"\.uses_dynamic_stack:\s+(\S+)", b)
        res.append((m.group(1), int(p.group(1)), d is not None and d.group(1) == "true"))
    return res


def test_no_kernel_uses_scratch(notes):
    n = 0
    for t, text in notes.items():
        ks = kernels(text)
        assert len(ks) > 40, (t, len(ks))
        bad = [(k, p, d) for k, p, d in ks if p or d]
        assert not bad, bad
        n += len(ks)
        names = " ".join(k for k, _, _ in ks)
        assert "rocprim" not in names and "cub" not in names.lower(), \
            "library kernels linked into the engine"
    assert n
