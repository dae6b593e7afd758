"""Register counts, LDS size and the s_waitcnt sequence of kernels in a built object (no GPU needed).

    python tools/isa_info.py <substring of the mangled kernel name> [object, default ppls_amd/_build/ppls_kernels.o]

Extracts the gfx950 code object from the object's .hip_fatbin section (objcopy + clang-offload-bundler),
then prints per matching kernel: VGPRs, AGPRs, spills, LDS bytes, the instruction counts that matter
for a streaming MFMA kernel and every s_waitcnt in program order.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    pat = sys.argv[1]
    obj = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..", "ppls_amd", "_build",
                                                             "ppls_kernels.o")
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                             text=True).stdout
    for m in re.finditer(r"\.name:\s+(\S+)", notes):
        name = m.group(1)
        if pat not in name or name.endswith(".kd"):
            continue
        # the metadata map of this kernel: from the previous list item to the next
        a = notes.rfind("\n  - ", 0, m.start())
        b = notes.find("\n  - ", m.end())
        blk = notes[a:b if b > 0 else len(notes)]

        def g(k):
            mm = re.search(r"\." + k + r":\s+(\d+)", blk)
            return int(mm.group(1)) if mm else None
        print(f"{name}: vgpr {g('vgpr_count')} agpr {g('agpr_count')} vgpr_spill {g('vgpr_spill_count')} "
              f"lds {g('group_segment_fixed_size')} scratch {g('private_segment_fixed_size')}")
        i = dis.find(f"<{name}>:")
        if i < 0:
            continue
        j = dis.find(">:\n", i + len(name) + 4)
        body = [ln.strip() for ln in dis[i:j if j > 0 else len(dis)].split("\n")[1:]]
        ins = [ln.split("//")[0].strip() for ln in body if ln and not ln.startswith("<")]
        c = collections.Counter(x.split()[0] for x in ins if x)
        keep = [k for k in c if k.startswith(("v_mfma", "global_load", "ds_read", "ds_write", "global_store",
                                              "s_barrier", "v_cvt", "buffer_"))]
        print("  " + ", ".join(f"{k} {c[k]}" for k in sorted(keep)))
        print("  waits: " + " | ".join(x.replace("s_waitcnt ", "") for x in ins if x.startswith("s_waitcnt")))


if __name__ == "__main__":
    main()
