"""Per-kernel fingerprint of the gfx950 machine code inside a built libwk.so: every code object of
the .hip_fatbin section unbundled (as kernel_resources.py does), disassembled, and each kernel's
instruction text hashed with addresses and branch offsets stripped.  Two builds whose kernels
hash the same run the same instructions -- the check that a source clean-up (dead build
options removed) left the product kernels unchanged.
usage: isa_fingerprint.py LIB [OTHER_LIB]   (one lib: print; two: diff)"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"


def code_objects(so, td):
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
        yield co


def fingerprints(so):
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for co in code_objects(so, td):
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                                  "--no-leading-addr", co], check=True, capture_output=True,
                                 text=True).stdout
            name, body = None, []
            for line in dis.splitlines() + ["<end>:"]:
                m = re.match(r"^(\S+) <(.+)>:$", line) or re.match(r"^<(.+)>:$", line)
                if m or line == "<end>:":
                    if name and body:
                        out[name] = (hashlib.sha1("\n".join(body).encode()).hexdigest()[:16], len(body))
                    name, body = (m.groups()[-1] if m else None), []
                    continue
                ins = line.strip()
                if not ins or ins.startswith(";"):
                    continue
                ins = re.sub(r"//.*$", "", ins).strip()
                ins = re.sub(r"<[^>]*>", "", ins)          # branch target labels
                ins = re.sub(r"0x[0-9a-f]+\b", "IMM", ins) if ins.startswith("s_cbranch") or \
                    ins.startswith("s_branch") else ins
                out_ins = ins
                body.append(out_ins)
    return out


if __name__ == "__main__":
    a = fingerprints(sys.argv[1])
    if len(sys.argv) == 2:
        for k, (h, n) in sorted(a.items()):
            print(f"{h} {n:6d} {k}")
        sys.exit(0)
    b = fingerprints(sys.argv[2])
    diff = 0
    for k in sorted(set(a) | set(b)):
        if a.get(k) != b.get(k):
            diff += 1
            print(f"DIFF {k}: {a.get(k)} -> {b.get(k)}")
    print(f"{len(set(a) & set(b))} kernels in both, {diff} differ")
    sys.exit(1 if diff else 0)
