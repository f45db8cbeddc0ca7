import re, sys
txt = open(sys.argv[1]).read().split('\n')
win = int(sys.argv[2]) if len(sys.argv) > 2 else 2
fn = None; hits = {}
for n, ln in enumerate(txt):
    if re.match(r'^[_A-Za-z][\w.]*:', ln) and not ln.startswith('.L'):
        fn = ln.split(':')[0]
    s = ln.strip()
    m = re.match(r'(buffer_store_dwordx[34]|global_store_dwordx[34]|flat_store_dwordx[34])\s', s)
    if not m: continue
    # data operand: buffer_store vdata, vaddr...; global_store vaddr, vdata
    if m.group(1).startswith('buffer'):
        d = re.match(r'\S+\s+v\[(\d+):(\d+)\]', s)
    else:
        d = re.match(r'\S+\s+\S+,\s*v\[(\d+):(\d+)\]', s)
    if not d: continue
    lo, hi = int(d.group(1)), int(d.group(2))
    k = 0; j = n + 1
    while k < win and j < len(txt):
        t = txt[j].strip(); j += 1
        if not t or t.startswith(';') or t.startswith('.'): continue
        k += 1
        op = t.split()[0]
        if op == 's_nop': 
            k += int(re.search(r's_nop\s+(\d+)', t).group(1)); continue
        if op.startswith('v_'):
            w = re.match(r'\S+\s+v\[(\d+):(\d+)\]', t)
            if w: a, b = int(w.group(1)), int(w.group(2))
            else:
                w = re.match(r'\S+\s+v(\d+)\b', t)
                if not w: continue
                a = b = int(w.group(1))
            if not (b < lo or a > hi):
                hits.setdefault(fn, []).append((n, s, t))
for f, h in hits.items():
    print(len(h), f[:110]); print('   ', h[0][1], ' -> ', h[0][2])
print("functions with hits:", len(hits))
