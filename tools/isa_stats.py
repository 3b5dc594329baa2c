#!/usr/bin/env python3
"""Static ISA statistics of one kernel in a `hipcc --offload-device-only -S` file.

    tools/isa_stats.py <file.s> <kernel-name-substring>

Prints the kernel's register / spill metadata and, for every innermost loop
(LLVM's "Loop Header" comments), the VALU / packed / SALU / LDS instruction
counts of the loop body (header .. last branch back to it).  A quick way to
compare code changes before spending a GPU run on them.
"""
import re
import sys


def main(path, key):
    text = open(path).read()
    lines = text.split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l]
    if not starts:
        sys.exit(f"no kernel matching {key}")
    s = starts[0]
    name = lines[s].split(":")[0]
    e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[s:e]
    # metadata block
    m = text.index(".name:           " + name)
    blk = text[m:m + 800]
    meta = dict(re.findall(r"\.(vgpr_count|vgpr_spill_count|sgpr_count|private_segment_fixed_size):\s+(\d+)", blk))
    print(name)
    print("  meta:", meta)
    cnt = lambda seg, p: sum(1 for l in seg if re.match(p, l.strip()))
    print("  total VALU %d  pk %d  SALU %d  LDS %d  scratch %d" % (
        cnt(body, r"v_"), cnt(body, r"v_pk_"), cnt(body, r"s_"), cnt(body, r"ds_"),
        cnt(body, r"scratch_")))
    # basic blocks: a label line carries LLVM's loop annotation
    # ("; in Loop: Header=BB7_32 Depth=2" / "; =>This Inner Loop Header: Depth=2")
    blocks, cur = [], None
    for i, l in enumerate(body):
        if re.match(r"^(\.LBB\S+|; %bb\.\d+):", l) or re.match(r"^; %bb\.\d+:", l):
            cur = [l]
            blocks.append(cur)
        elif cur is not None:
            cur.append(l)
    for bi, b in enumerate(blocks):
        if not any("Inner Loop Header" in x for x in b[:3]):
            continue
        lab = b[0].split(":")[0].lstrip(".")  # LBB204_32
        hid = lab.replace("LBB", "BB")
        seg = list(b)
        for b2 in blocks[bi + 1:]:
            if "Header=" + hid + " " in b2[0] or "Header=" + hid + "\t" in b2[0] or b2[0].rstrip().endswith("Header=" + hid):
                seg += b2
            elif re.search(r"Header=" + hid + r"\b", b2[0]):
                seg += b2
        depth = re.search(r"Depth=(\d+)", " ".join(b[:3])).group(1)
        print("  loop %s (depth %s, %d lines): VALU %d  pk %d  mov/cndmask %d  SALU %d  LDS %d  scratch %d" % (
            lab, depth, len(seg), cnt(seg, r"v_"), cnt(seg, r"v_pk_"),
            cnt(seg, r"v_(mov|cndmask)"), cnt(seg, r"s_"), cnt(seg, r"ds_"), cnt(seg, r"scratch_")))

if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
