"""The built library's gfx950 code objects (CPU only: reads liblqro.so's
kernel descriptors, runs nothing).

Guards what the kernel metadata shows and a timing run would not: k_dynw keeps
no private (scratch) memory — its device functions are inlined and the 3x3
pivot permutations are packed into one integer — and k_qhull's
LDS fits one CU (160 KB).
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lqr-obstacles_amd", "liblqro.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tools():
    need = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not os.path.exists(LIB) or not all(os.path.exists(t) for t in need):
        pytest.skip("liblqro.so or the ROCm LLVM tools are missing")


def _kernels():
    """{kernel name: {metadata key: int}} over every gfx950 code object in the library."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fatbin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, LIB],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
        assert starts, "no offload bundle in .hip_fatbin"
        for n, s in enumerate(starts):
            e = starts[n + 1] if n + 1 < len(starts) else len(blob)
            b = os.path.join(d, "b%d" % n)
            with open(b, "wb") as fh:
                fh.write(blob[s:e])
            co = b + ".gfx950.o"
            r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + b,
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co],
                               capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            # one kernel's metadata: a "- .args:" list entry; keys follow it
            for block in notes.split("\n  - .")[1:]:
                name = re.search(r"\.name:\s+(\S+)", block)
                if not name:
                    continue
                meta = {k: int(v) for k, v in re.findall(r"\.(\w+):\s+(\d+)\s*$", block, re.M)}
                out[name.group(1)] = meta
    return out


def test_dynw_no_scratch_qhull_lds_fits():
    _tools()
    ks = _kernels()
    dynw = [k for k in ks if "k_dynw" in k]
    qhull = [k for k in ks if re.search(r"7k_qhull", k)]
    assert dynw and qhull, sorted(ks)[:20]
    for k in dynw:
        assert ks[k].get("private_segment_fixed_size", -1) == 0, (k, ks[k])
    for k in qhull:
        assert 0 < ks[k].get("group_segment_fixed_size", 0) <= 160 * 1024, (k, ks[k])
