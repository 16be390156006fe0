"""Instruction mix of kernels and of their loops in a device assembly file (hipcc
--cuda-device-only -S): python tools/isa_stats.py file.s name_substring [...]. A loop is the set
of basic blocks the compiler annotates with the same loop header."""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@", text, re.M):
        end = text.find(".Lfunc_end", m.end())
        yield m.group(1), text[m.end():end]


def mix(lines):
    ops = {}
    for l in lines:
        op = l.split()[0]
        ops[op] = ops.get(op, 0) + 1

    def cnt(f):
        return sum(v for k, v in ops.items() if f(k))
    return dict(n=len(lines), mfma=cnt(lambda k: "mfma" in k), valu=cnt(lambda k: k.startswith("v_") and "mfma" not in k),
                salu=cnt(lambda k: k.startswith("s_") and not k.startswith(("s_load", "s_waitcnt", "s_cbranch", "s_branch", "s_nop", "s_barrier"))),
                ds=cnt(lambda k: k.startswith("ds_")), vmem=cnt(lambda k: k.startswith(("global_", "buffer_"))),
                scratch=cnt(lambda k: k.startswith("scratch_")), s_load=cnt(lambda k: k.startswith("s_load")),
                waitcnt=ops.get("s_waitcnt", 0), exp=cnt(lambda k: k.startswith("v_exp")),
                cndmask=cnt(lambda k: k.startswith("v_cndmask")))


def main():
    text = open(sys.argv[1]).read()
    for name, body in kernels(text):
        if not any(s in name for s in sys.argv[2:]):
            continue
        blocks, cur, hdr = [], [], None
        for raw in body.split("\n"):
            st = raw.strip()
            m = re.match(r"(\.LBB\d+_\d+):(.*)", st)
            if m:
                blocks.append((hdr, cur))
                cur = []
                h = re.search(r"Header=BB(\d+_\d+)", m.group(2))
                hdr = ".LBB" + h.group(1) if h else (m.group(1) if "Loop Header" in m.group(2) else None)
                continue
            l = st.split(";")[0].strip()
            if l and not l.startswith("."):
                cur.append(l)
        blocks.append((hdr, cur))
        print(name, mix([l for _, b in blocks for l in b]))
        for h in sorted({h for h, _ in blocks if h}):
            m = mix([l for hh, b in blocks if hh == h for l in b])
            if m["mfma"]:
                print("   loop", h, m)


if __name__ == "__main__":
    main()
