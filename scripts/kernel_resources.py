"""Register / scratch use of the kernels in a hipcc object (its gfx950 code object's metadata notes).

    python scripts/kernel_resources.py stochastic-epidemic-modelling_amd/lib/epipf_group.o [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj = os.path.abspath(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as d:
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", obj], cwd=d, capture_output=True, check=True)
        cos = [f for f in os.listdir(os.path.dirname(obj)) if f.startswith(os.path.basename(obj) + ".0.hipv4")]
        co = os.path.join(os.path.dirname(obj), cos[0])
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        for f in cos:
            os.remove(os.path.join(os.path.dirname(obj), f))
        for f in os.listdir(os.path.dirname(obj)):
            if f.startswith(os.path.basename(obj) + ".0.host"):
                os.remove(os.path.join(os.path.dirname(obj), f))
    keys = ["private_segment_fixed_size", "sgpr_count", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count"]
    for blk in notes.split("  - .")[1:]:
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or filt not in m.group(1):
            continue
        vals = {k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "?"])[1] for k in keys}
        print(m.group(1), " ".join(f"{k.replace('_count', '').replace('private_segment_fixed_size', 'scratch')}={v}"
                                   for k, v in vals.items()))


if __name__ == "__main__":
    main()
