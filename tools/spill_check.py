"""Register spills of the library's kernels, from the code objects in libneo_hip.so (no GPU, no
compile): the .hip_fatbin section's offload bundles -> the gfx950 ELF of every translation unit ->
its AMDGPU metadata note (llvm-readelf --notes): per kernel .vgpr_count, .vgpr_spill_count,
.sgpr_spill_count, .private_segment_fixed_size. Prints JSON; tests/test_abi.py asserts that the
hot kernels spill nothing (a second inlined copy of the slice roles once spilled 104 VGPRs in
k_lvl_slices and cost the c5full step 12 %)."""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so_path):
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", so_path,
                        os.path.join(d, "x.so")], check=True, capture_output=True)
        blob = open(fb, "rb").read()
    out = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                out.append(blob[pos + off:pos + off + size])
        pos = blob.find(MAGIC, pos + 1)
    return out


def kernels(so_path):
    res = {}
    for co in code_objects(so_path):
        with tempfile.NamedTemporaryFile(suffix=".o") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], capture_output=True,
                                 text=True).stdout
        for block in txt.split("  - .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", block)
            if not name:
                continue
            get = lambda k: int(re.search(rf"{k}:\s+(\d+)", block).group(1)) if re.search(rf"{k}:\s+(\d+)", block) else None
            res[name.group(1)] = {"vgpr": get(r"\.vgpr_count"), "vgpr_spill": get(r"\.vgpr_spill_count"),
                                  "sgpr_spill": get(r"\.sgpr_spill_count"), "scratch": get(r"\.private_segment_fixed_size")}
    return res


if __name__ == "__main__":
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "neo-dsp_amd", "lib", "libneo_hip.so")
    print(json.dumps(kernels(so), indent=1))
