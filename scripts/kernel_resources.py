"""Per-kernel VGPR / AGPR / SGPR / scratch / LDS of one object in deepflame-dev_amd/csrc/build, read from the
gfx950 code object's metadata notes. Usage: python scripts/kernel_resources.py chem.hip.o [kernel-name-regex]"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
obj = sys.argv[1] if os.path.sep in sys.argv[1] else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "deepflame-dev_amd", "csrc", "build", sys.argv[1])
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
with tempfile.TemporaryDirectory() as d:
    fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "dev.co")
    subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj], check=True)
    subprocess.run([f"{B}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={fb}", f"--output={co}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
    txt = subprocess.run([f"{B}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
for blk in txt.split("- .agpr_count")[1:]:
    def g(k):
        m = re.search(r"\.%s:\s+(\S+)" % k, blk)
        return m.group(1) if m else "?"
    agpr = blk.split("\n", 1)[0].strip(": ")
    name = g("name")
    if not pat.search(name):
        continue
    print("%-100s vgpr %4s agpr %4s sgpr %4s scratch %5s lds %6s" % (name[:100], g("vgpr_count"), agpr,
          g("sgpr_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size")))
