"""Per-kernel scratch (private segment bytes) and VGPR spill counts of the gfx950 code objects
inside a built libwk.so: the .hip_fatbin section is split at each offload bundle, the gfx950
object of each unbundled, and the AMDHSA metadata notes read.  usage: kernel_resources.py [lib]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_resources(so):
    """{kernel symbol: (private_segment_fixed_size, vgpr_spill_count, vgpr_count)}"""
    res = {}
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so,
                        os.path.join(td, "stripped")], check=True, capture_output=True)
        data = open(fat, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
        for i, o in enumerate(offs):
            p, co = os.path.join(td, f"b{i}.bin"), os.path.join(td, f"b{i}.o")
            with open(p, "wb") as f:
                f.write(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={p}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                           check=True, capture_output=True)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)
                ps = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1))
                vs = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1))
                vc = int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1))
                res[name] = (ps, vs, vc)
    return res


if __name__ == "__main__":
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "ppo-bipedalwalker_amd", "libwk.so")
    for k, (ps, vs, vc) in sorted(kernel_resources(so).items()):
        print(f"{ps:5d} B scratch  {vs:4d} spilled  {vc:4d} VGPRs  {k}")
