"""Per-kernel load / wait / MFMA order from a device assembly listing (round 3).

Build the listing on the CPU:
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude --cuda-device-only -S \
      llmvox_amd/csrc/ar_kernels.hip -o /tmp/ar.s
then
  python tools/isa_loadseq.py /tmp/ar.s ar_rows_kernelILi4 ar_embed_select ...
prints, for every kernel whose mangled name contains one of the patterns, its sequence of global /
buffer loads (L<n>: n loads in a row), `s_waitcnt vmcnt(k)` (w<k>) and MFMAs (M<n>) up to s_endpgm.
A kernel meant to have every load in flight before its first use shows one L run before the first
wait; `L12 w8 L3` means 3 loads were issued only after the first ones landed (one more dependent
round trip)."""
import re
import sys


def main(path, pats):
    asm = open(path).read().split("\n")
    for i, line in enumerate(asm):
        m = re.match(r"^(_ZN3lvx\S+):", line)
        if not m or not any(p in m.group(1) for p in pats):
            continue
        seq = []
        for body in asm[i + 1:i + 4000]:
            if "s_endpgm" in body:
                break
            if re.search(r"\b(global_load|buffer_load)", body):
                seq.append("L")
            elif "s_waitcnt" in body and "vmcnt" in body:
                seq.append("w" + re.search(r"vmcnt\((\d+)\)", body).group(1))
            elif "v_mfma" in body:
                seq.append("M")
        s = " ".join(seq) + " "
        s = re.sub(r"(L )+", lambda r: f"L{r.group(0).count('L')} ", s)
        s = re.sub(r"(M )+", lambda r: f"M{r.group(0).count('M')} ", s)
        print(m.group(1)[:100])
        print("   ", s.strip()[:400])


if __name__ == "__main__":
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    main(sys.argv[1], sys.argv[2:])
