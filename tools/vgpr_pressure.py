#!/usr/bin/env python3
"""VGPR liveness over a kernel's gfx950 assembly (hipcc -S): backward dataflow on the basic
blocks, then the instructions with the most live VGPRs (where the allocator ran out and had
to spill).  Usage: tools/vgpr_pressure.py FILE.s KERNEL_SYMBOL_SUBSTRING [--top N] [--ctx C]"""
import argparse
import re

RX = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
# instructions whose first operand is not a VGPR definition
NODEF = ("v_cmp_", "v_cmpx_", "ds_write", "ds_store", "global_store", "scratch_store",
         "buffer_store", "flat_store", "s_", "v_readlane", "v_readfirstlane", "ds_swizzle_nop")


def vregs(tok):
    out = []
    for m in RX.finditer(tok):
        if m.group(3):
            out.append(int(m.group(3)))
        else:
            out += range(int(m.group(1)), int(m.group(2)) + 1)
    return out


def parse(lines):
    insts = []  # (lineno, text, op, defs, uses, label or None, branch target, cond)
    for i, l in enumerate(lines):
        t = l.split(";")[0].rstrip()
        s = t.strip()
        if not s:
            continue
        if re.match(r"^[.\w$]+:$", s):
            insts.append(dict(ln=i, label=s[:-1]))
            continue
        if s.startswith("."):
            continue
        parts = s.split(None, 1)
        op = parts[0]
        args = [a.strip() for a in parts[1].split(",")] if len(parts) > 1 else []
        defs, uses = [], []
        if args and not op.startswith(NODEF) and not op.startswith("v_cmp"):
            defs = vregs(args[0])
            for a in args[1:]:
                uses += vregs(a)
            # partial writes (sdwa / dpp / cndmask with old value) are treated as full defs
        else:
            for a in args:
                uses += vregs(a)
            if op.startswith("v_readlane") or op.startswith("v_readfirstlane"):
                pass
            if op.startswith("v_cmp") and not op.startswith("v_cmpx"):
                pass
        tgt = None
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = args[0] if args else None
        insts.append(dict(ln=i, op=op, text=s, defs=set(defs), uses=set(uses), tgt=tgt))
    return insts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--ctx", type=int, default=0)
    ap.add_argument("--who", action="store_true",
                    help="for the peak, each live register's nearest preceding definition")
    a = ap.parse_args()
    lines = open(a.asm).read().split("\n")
    st = next(i for i, l in enumerate(lines) if a.kernel in l
              and l.split(";")[0].rstrip().endswith(":") and not l.startswith("."))
    en = next(i for i in range(st, len(lines)) if "s_endpgm" in lines[i])
    ins = parse(lines[st:en + 1])
    # basic blocks
    blocks, cur = [], []
    for x in ins:
        if "label" in x:
            if cur:
                blocks.append(cur)
            cur = [x]
        else:
            cur.append(x)
            if "tgt" in x and x["tgt"] is not None:
                blocks.append(cur)
                cur = []
    if cur:
        blocks.append(cur)
    lab = {}
    for bi, b in enumerate(blocks):
        for x in b:
            if "label" in x:
                lab[x["label"]] = bi
    succ = []
    for bi, b in enumerate(blocks):
        s = []
        last = next((x for x in reversed(b) if "op" in x), None)
        if last is not None and last.get("tgt"):
            if last["tgt"] in lab:
                s.append(lab[last["tgt"]])
            if last["op"] != "s_branch" and bi + 1 < len(blocks):
                s.append(bi + 1)
        elif last is not None and last["op"] == "s_endpgm":
            pass
        elif bi + 1 < len(blocks):
            s.append(bi + 1)
        succ.append(s)
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for bi in reversed(range(len(blocks))):
            out = set()
            for s in succ[bi]:
                out |= live_in[s]
            live = set(out)
            for x in reversed(blocks[bi]):
                if "op" in x:
                    live -= x["defs"]
                    live |= x["uses"]
            if live != live_in[bi]:
                live_in[bi] = live
                changed = True
    # per-instruction live-out counts
    rec = []
    for bi, b in enumerate(blocks):
        out = set()
        for s in succ[bi]:
            out |= live_in[s]
        live = set(out)
        for x in reversed(b):
            if "op" in x:
                rec.append((len(live | x["defs"]), x["ln"] + st, x["text"], frozenset(live)))
                live -= x["defs"]
                live |= x["uses"]
    rec.sort(key=lambda r: -r[0])
    print(f"max live VGPRs {rec[0][0]}; instructions at >= max-4: "
          f"{sum(1 for r in rec if r[0] >= rec[0][0] - 4)}")
    seen = set()
    for n, ln, text, live in rec:
        if len(seen) >= a.top:
            break
        if any(abs(ln - s) < 40 for s in seen):
            continue
        seen.add(ln)
        print(f"-- {n} live at line {ln - st}: {text}")
        if a.ctx:
            for j in range(ln - a.ctx, ln + a.ctx + 1):
                print(f"   {j - st}: {lines[j].strip()[:110]}")
        if a.who and len(seen) == 1:
            defs = [(x["ln"], x) for x in ins if "op" in x and x["defs"]]
            for r in sorted(live):
                d = [(l_, x) for l_, x in defs if r in x["defs"] and l_ < ln]
                l_, x = d[-1] if d else (None, None)
                print(f"   v{r}: def at {l_} {x['text'][:70] if x else '?'}")


if __name__ == "__main__":
    main()
