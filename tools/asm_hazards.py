"""Scan gfx950 device assembly (hipcc --cuda-device-only -S) for inline-asm VALU instructions placed
within the MFMA dependency windows that LLVM's hazard recognizer does not check for inline asm
(GCNHazardRecognizer::checkInlineAsmHazards covers neither the XDL->VALU RAW/WAR windows nor
VALU->XDL reads). Reports, per kernel symbol, inline-asm v_max_f32 (cnf_device.h lrelu) that
  RAW  reads a VGPR an MFMA wrote fewer than `win` wait states earlier,
  WAR  writes a VGPR an in-flight MFMA reads as SrcC (fewer than `win` wait states since its issue),
  FWD  writes a VGPR an MFMA reads within 2 wait states after it.
Wait states are counted as issued instructions (s_nop N counts N + 1); the window is the 16-pass
worst case. usage: python tools/asm_hazards.py file.s [win]
       python tools/asm_hazards.py --overlap file.s   MFMAs whose vdst partially overlaps srcC, per kernel
(hipcc's allocation of some bf16x6 chains in k_pw / k_gc)
Compiler-scheduled instructions that read an MFMA's result or write its SrcC retire its window (the
compiler padded them). Diagnostic only: the round-6 nondeterminism was not explained by either finding."""
import re
import sys

REG = re.compile(r'\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b')


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
            out |= {(k, i) for i in range(a, b + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def parse(line):
    s = line.split(';')[0].strip()
    if not s or s.endswith(':') or s.startswith('.'):
        return None
    op, _, rest = s.partition(' ')
    ops = [o.strip() for o in rest.split(',')] if rest else []
    return op, ops


def overlap(path):
    sym, per = '?', {}
    for line in open(path):
        t = line.strip()
        m = re.match(r'^(_Z\w+):', t)
        if m:
            sym = m.group(1)
            continue
        if t.startswith('v_mfma'):
            p = parse(t)
            if p is None or len(p[1]) < 4:
                continue
            d, c = regs(p[1][0]), regs(p[1][3])
            if d & c and d != c:
                per[sym] = per.get(sym, 0) + 1
    for k, v in sorted(per.items()):
        print(f'{v:4d} {k}')
    print(f'{sum(per.values())} partial vdst/srcC overlaps in {len(per)} kernels', file=sys.stderr)


def main():
    if sys.argv[1] == '--overlap':
        overlap(sys.argv[2])
        return
    path = sys.argv[1]
    win = int(sys.argv[2]) if len(sys.argv) > 2 else 18
    sym = '?'
    hist = []   # (ws_index, op, ops, is_asm)
    ws = 0
    in_asm = False
    hits = {}
    where = {}
    pending_fwd = []   # (ws, dst regs, sym)
    for lno, line in enumerate(open(path), 1):
        t = line.strip()
        if re.match(r'^[A-Za-z_.$][\w.$]*:\s*(;.*)?$', t) and not t.startswith('.L'):
            sym = t.split(':')[0]
            hist, pending_fwd = [], []
            continue
        if ';;#ASMSTART' in t:
            in_asm = True
            continue
        if ';;#ASMEND' in t:
            in_asm = False
            continue
        p = parse(t)
        if p is None:
            continue
        op, ops = p
        n = 1
        if op == 's_nop' and ops:
            n = int(ops[0], 0) + 1
        if op.startswith('v_mfma'):
            dst, srcs = regs(ops[0]), [regs(o) for o in ops[1:4]]
            for (w0, dregs, s0) in pending_fwd:
                if ws - w0 < 2 and any(dregs & s for s in srcs):
                    hits.setdefault((s0, 'FWD'), 0)
                    hits[(s0, 'FWD')] += 1
            # a later MFMA chained on the same accumulator supersedes the earlier entry
            hist = [h for h in hist if not (h[2] & dst)]
            # WAR window: SrcC only (SrcA/B are read at issue)
            hist.append((ws, 'mfma', dst, srcs[2] if len(srcs) > 2 else set()))
        elif not in_asm and ops:
            # a compiler-scheduled instruction reading an MFMA result waited for it: that MFMA retired
            rd = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
            if op.startswith(('buffer_store', 'global_store', 'ds_write', 'flat_store')):
                rd |= set().union(*[regs(o) for o in ops])
            hist = [h for h in hist if not (h[2] & rd)]
            if not op.startswith(('buffer_store', 'global_store', 'ds_write', 'flat_store', 's_')):
                wr = regs(ops[0])   # overwritten: no longer the MFMA's result
                # a compiler VALU write into an MFMA's SrcC waited out that MFMA's WAR window
                wv = op.startswith('v_') and not op.startswith('v_mfma')
                hist = [(h[0], h[1], h[2] - wr, set() if (wv and h[3] & wr) else h[3]) for h in hist]
        if in_asm and op.startswith('v_'):
            dregs = regs(ops[0]) if ops else set()
            sregs = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
            for (w0, kind, mdst, msrc) in hist:
                if kind != 'mfma' or ws - w0 >= win:
                    continue
                if sregs & mdst:
                    hits[(sym, 'RAW')] = hits.get((sym, 'RAW'), 0) + 1
                    where.setdefault((sym, 'RAW'), lno)
                if dregs & msrc:
                    hits[(sym, 'WAR')] = hits.get((sym, 'WAR'), 0) + 1
                    where.setdefault((sym, 'WAR'), lno)
            pending_fwd.append((ws, dregs, sym))
            pending_fwd = pending_fwd[-8:]
        ws += n
        hist = [h for h in hist if ws - h[0] < win]
    for (s, k), c in sorted(hits.items()):
        print(f'{k} {c:4d} {s} (first at line {where.get((s, k))})')
    print(f'{len(hits)} (kernel, kind) pairs with hazards', file=sys.stderr)


if __name__ == '__main__':
    main()
