"""Static check of hand-placed vmcnt waits in a gfx950 kernel (tuning aid).

Walks the assembly of one kernel linearly (a loop body is seen once per pass;
run with --passes 2 to model one back-edge), keeps the in-order queue of
outstanding VMEM operations, retires entries at every `s_waitcnt vmcnt(N)`,
and reports any instruction that reads or overwrites a VGPR that is still the
destination of an outstanding load -- the hazard of issuing loads from inline
asm, where the compiler does not insert waits itself.
    python tools/check_vmcnt.py kernels.s _ZN8lssp_amd9k_tri_pk6ILi4ELi2ELb0ELi256EEEvNS_7Pk6ArgsE
"""
import re
import sys

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main(path, name, passes=2):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = [l.split(";")[0].strip() for l in lines[start:end]]
    body = [l for l in body if l and not l.endswith(":") and not l.startswith(".")]
    queue = []  # [(dest regs or empty set, index)]
    issues = 0
    for p in range(passes):
        for i, ins in enumerate(body):
            op = ins.split()[0]
            args = ins[len(op):]
            m = re.match(r"s_waitcnt\s+vmcnt\((\d+)\)", ins)
            if m or (op == "s_waitcnt" and "vmcnt" in ins):
                n = int(re.search(r"vmcnt\((\d+)\)", ins).group(1))
                while len(queue) > n:
                    queue.pop(0)
                continue
            parts = [x.strip() for x in args.split(",")]
            is_vmem = op.startswith(("global_", "buffer_", "flat_", "scratch_"))
            if is_vmem and "load" in op and "lds" not in op:
                dst, src = regs(parts[0]), regs(",".join(parts[1:]))
            elif is_vmem:
                dst, src = set(), regs(args)
            elif op.startswith(("v_", "ds_")) and parts and parts[0]:
                if op.startswith("ds_write") or op.startswith("ds_store"):
                    dst, src = set(), regs(args)
                else:
                    dst, src = regs(parts[0]), regs(",".join(parts[1:]))
            else:
                dst, src = set(), regs(args)
            pending = set().union(*[q[0] for q in queue]) if queue else set()
            bad = (src | dst) & pending
            if bad and p == passes - 1:
                issues += 1
                if issues <= 20:
                    print(f"hazard: {ins}   (pending v{sorted(bad)})")
            if is_vmem:
                queue.append((dst, i))
    print(f"{name}: {issues} hazards")
    return issues


def check_loader(path, name, repeat=3):
    """Check the inline-asm loader loop of a k_tri_pk6 instantiation: the
    region from its first asm index load to the vmcnt(0) after the loop,
    unrolled `repeat` times to model the back-edge.  Returns the hazard count."""
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    en = next(i for i in range(st, len(lines)) if "s_endpgm" in lines[i])
    seg = lines[st:en]
    idx = [i for i, l in enumerate(seg) if re.match(r"\s*global_load_dword v\d+, v\[\d+:\d+\], off$", l)]
    a = max(idx[0] - 5, 0)
    b = max(i for i, l in enumerate(seg) if "s_waitcnt vmcnt(0)" in l and i > idx[-1])
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".s", delete=False) as f:
        f.write(name + ":\n" + "\n".join(seg[a:b] * repeat) + "\n\ts_endpgm\n")
    return main(f.name, name, passes=1)


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1], sys.argv[2]) else 0)
