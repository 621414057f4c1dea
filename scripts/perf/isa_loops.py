"""Static instruction mix of a kernel's loops from a `hipcc -S` listing: splits the named kernel into basic blocks,
finds back edges (a branch to an earlier label), and prints, per loop, the instruction count by class -- the
per-iteration issue budget the PMC's VALU / SALU / LDS counts come from.

    python scripts/perf/isa_loops.py villain_hot.s _ZN2sv17villain_sweep_hotILb0ELi4EEEvNS_5FArgsE"""
import collections
import re
import sys

path, kern = sys.argv[1], sys.argv[2]
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if l.startswith(kern + ':'))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith('s_endpgm'))
body = lines[start:end + 1]
labels = {}
insts = []  # (index, label or None, mnemonic, text)
for l in body:
    s = l.split(';')[0].strip()
    if not s:
        continue
    m = re.match(r'^(\.LBB\S+):', s)
    if m:
        labels[m.group(1)] = len(insts)
        continue
    if s.startswith('.'):
        continue
    insts.append((s.split()[0], s))


def klass(mn):
    if mn.startswith('v_mfma'):
        return 'mfma'
    if mn.startswith('ds_'):
        return 'lds'
    if mn.startswith(('global_', 'buffer_', 'flat_')):
        return 'vmem'
    if mn.startswith('scratch_'):
        return 'scratch'
    if mn.startswith('s_waitcnt') or mn.startswith('s_barrier'):
        return 'wait/barrier'
    if mn.startswith(('s_cbranch', 's_branch')):
        return 'branch'
    if mn.startswith('s_'):
        return 'salu'
    if mn.startswith('v_'):
        if '_f64' in mn:
            return 'valu_f64'
        if any(k in mn for k in ('_u64', '_i64', 'lshlrev_b64', 'lshrrev_b64', 'ashrrev_i64', 'mad_u64', 'mad_i64')):
            return 'valu_64int'
        return 'valu_32'
    return 'other'


loops = []
for i, (mn, s) in enumerate(insts):
    if mn.startswith(('s_cbranch', 's_branch')):
        tgt = s.split()[-1]
        if tgt in labels and labels[tgt] <= i:
            loops.append((labels[tgt], i))
for a, b in sorted(loops, key=lambda x: x[1] - x[0], reverse=True)[:4]:
    c = collections.Counter(klass(insts[k][0]) for k in range(a, b + 1))
    mns = collections.Counter(insts[k][0] for k in range(a, b + 1) if insts[k][0].startswith('v_'))
    print(f'loop [{a}, {b}] {b - a + 1} instructions: ' + ', '.join(f'{k} {v}' for k, v in c.most_common()))
    print('   top VALU: ' + ', '.join(f'{k} {v}' for k, v in mns.most_common(25)))
print(f'kernel: {len(insts)} instructions, ' + ', '.join(f'{k} {v}' for k, v in collections.Counter(klass(m) for m, _ in insts).most_common()))
