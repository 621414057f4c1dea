"""Attribute a kernel's main-loop instructions to the source functions they were inlined from.

Compiles nothing: reads a `hipcc -g -S` listing (the -g only adds .loc lines; the ISA is the same), takes the kernel's
largest loops (back edges, as isa_loops.py), and charges every instruction to the innermost function or named lambda
whose source range holds the instruction's .loc line (brace matching over the source files).  Prints, per loop, the
VALU / LDS / memory / scalar counts per source function and per category.

    python scripts/perf/isa_attrib.py /tmp/vhg.s _ZN2sv17villain_sweep_hotILb0ELi4EEEvNS_5FArgsE [loops]"""
import collections
import os
import re
import sys

path, kern = sys.argv[1], sys.argv[2]
nloops = int(sys.argv[3]) if len(sys.argv) > 3 else 2
lines = open(path).read().split('\n')
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
    if m:
        d, f = m.group(2), m.group(3)
        files[int(m.group(1))] = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(path)) if d == '.' else d, f)) \
            if not d.startswith('/') else os.path.join(d, f)
src_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'supervillain_amd', 'csrc')
for k, v in list(files.items()):  # (relative .file entries: the library's sources)
    cand = os.path.join(src_dir, os.path.basename(v))
    if os.path.exists(cand) and not v.startswith(('/usr', '/opt')):
        files[k] = cand

start = next(i for i, l in enumerate(lines) if l.startswith(kern + ':'))
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end') and i > start)
labels, insts = {}, []  # insts: (mnemonic, text, (file, line))
loc = (None, 0)
for l in lines[start:end]:
    s = l.split(';')[0].strip()
    if not s:
        continue
    m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
    if m:
        loc = (int(m.group(1)), int(m.group(2)))
        continue
    m = re.match(r'^(\.LBB\S+):', s)
    if m:
        labels[m.group(1)] = len(insts)
        continue
    if s.startswith('.'):
        continue
    insts.append((s.split()[0], s, loc))


# source ranges of functions and named lambdas, per file: [(first, last, name)]
def ranges(fname):
    try:
        text = open(fname).read().split('\n')
    except OSError:
        return []
    out = []
    for i, l in enumerate(text):
        m = re.search(r'auto\s+(\w+)\s*=\s*\[', l)
        name = m.group(1) if m else None
        if name is None and re.search(r'__device__|__global__|__host__|SV_HD', l):
            m = re.search(r'\b(\w+)\s*\((?!.*;\s*$)', l.split('//')[0])
            name = m.group(1) if m else None
        if not name or name in ('if', 'for', 'while', 'switch', 'launch_bounds', '__launch_bounds__', 'attribute',
                                '__attribute__', 'amdgpu_waves_per_eu', 'sizeof'):
            continue
        # the body: first '{' at or after this line, to its matching '}'
        depth, opened, j = 0, False, i
        while j < len(text):
            seg = text[j].split('//')[0]
            for ch in seg:
                if ch == '{':
                    depth += 1
                    opened = True
                elif ch == '}':
                    depth -= 1
            if opened and depth <= 0:
                break
            if not opened and seg.rstrip().endswith(';'):
                break
            j += 1
        if opened:
            out.append((i + 1, j + 1, name))
    return out


RANGES = {}


def owner(loc):
    f, line = loc
    if f is None:
        return '?'
    fname = files.get(f, '?')
    if fname not in RANGES:
        RANGES[fname] = ranges(fname)
    best = None
    for a, b, name in RANGES[fname]:
        if a <= line <= b and (best is None or b - a < best[1] - best[0]):
            best = (a, b, name)
    base = os.path.basename(fname)
    return f'{base}:{best[2]}' if best else f'{base}:{line}'


def klass(mn):
    if mn.startswith('ds_'):
        return 'lds'
    if mn.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
        return 'vmem'
    if mn.startswith(('s_waitcnt', 's_barrier')):
        return 'wait'
    if mn.startswith('s_'):
        return 'salu'
    if mn.startswith('v_'):
        return 'valu64' if re.search(r'_f64|_u64|_i64|_b64', mn) else 'valu'
    return 'other'


CATEGORY = [  # (substring of the owner, category)
    ('mad_kk', 'PCG64 composition'), ('mad_k', 'PCG64 composition'), ('mad_n', 'PCG64 composition'),
    ('fma3', 'exp'), ('base_pos', 'row-base advance'), ('wrapN', 'index wrap (wrapN)'), ('jump', 'row-base advance'),
    ('hot_apply', 'PCG64 composition'), ('mad128', 'PCG64 composition'), ('apply', 'PCG64 composition'),
    ('compose', 'PCG64 composition'), ('xsl_rr', 'XSL-RR output'), ('u53', 'u53 / uniform'),
    ('to_double', 'u53 / uniform'), ('exp_ocml', 'exp'), ('sv_exp', 'exp'), ('lemire', 'Lemire'),
    ('fx_add', 'statistics (exact sums)'), ('flush_stats', 'statistics (exact sums)'), ('ballot', 'ballot'),
    ('hot_draws', 'draw words (pairing / DPP)'), ('fast_pack', 'draw words (pairing / DPP)'),
    ('store_rows', 'HBM row stores'), ('load_rows', 'HBM row loads'), ('commit', 'row commit'),
    ('prefetch', 'HBM row loads'), ('advance', 'row-base advance'), ('full_jump', 'row-base advance'),
]


def category(own):
    for key, cat in CATEGORY:
        if key in own.split(':')[-1]:
            return cat
    return own


# natural loops from the compiler's block annotations ("Loop: Header=BBx" / "Loop Header"): the row loops of the
# kernel's bodies are the two largest (interior strips and edge strips)
blocks, cur, loc = [], None, (None, 0)
for l in lines[start:end]:
    s = l.split(';')[0].strip()
    m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
    if m:
        loc = (int(m.group(1)), int(m.group(2)))
        continue
    m = re.match(r'^(\.LBB\S+):', s)
    if m:
        mm = re.search(r'Loop: Header=(\S+)', l)
        h = mm.group(1) if mm else ('BB' + m.group(1)[4:] if 'Loop Header' in l else None)
        cur = [m.group(1), h, []]
        blocks.append(cur)
        continue
    if not s or s.startswith('.') or cur is None:
        continue
    cur[2].append((s.split()[0], s, loc))
sizes = collections.Counter()
for b in blocks:
    if b[1]:
        sizes[b[1]] += len(b[2])
for H, n in sizes.most_common(nloops):
    per = collections.defaultdict(collections.Counter)
    cat = collections.defaultdict(collections.Counter)
    tot = collections.Counter()
    rare = collections.Counter()
    for b in blocks:
        if b[1] != H:
            continue
        is_rare = any(owner(lc).endswith(':report') or mn.startswith('global_atomic') for mn, _, lc in b[2])
        for mn, s, lc in b[2]:
            o, k = owner(lc), klass(mn)
            tot[k] += 1
            if is_rare:
                rare[k] += 1
                continue
            per[o][k] += 1
            cat[category(o)][k] += 1
    print(f'loop {H}: {n} instructions: ' + ', '.join(f'{k} {v}' for k, v in sorted(tot.items())) +
          f'; in blocks that report a rejection (rare): ' + ', '.join(f'{k} {v}' for k, v in sorted(rare.items())))
    print('  by category, common blocks (valu + valu64 | lds | vmem | salu):')
    for c, cnt in sorted(cat.items(), key=lambda kv: -(kv[1]['valu'] + kv[1]['valu64'])):
        print(f'    {c:44s} {cnt["valu"] + cnt["valu64"]:5d} ({cnt["valu64"]:4d} 64-bit) | {cnt["lds"]:4d} | '
              f'{cnt["vmem"]:3d} | {cnt["salu"]:4d}')
