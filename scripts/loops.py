# Developer tool: loop-by-loop instruction counts of one kernel in a hipcc --save-temps .s file.
import re,sys,subprocess
asm=open(sys.argv[1]).read()
kern=sys.argv[2]
m=re.search(r'^'+re.escape(kern)+r':.*?^\.Lfunc_end', asm, re.S|re.M)
body=m.group(0).splitlines()
# find loops: backward branches to a label
labels={}
for i,l in enumerate(body):
    mm=re.match(r'^(\.LBB\d+_\d+):',l)
    if mm: labels[mm.group(1)]=i
for i,l in enumerate(body):
    mm=re.search(r's_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)',l)
    if mm:
        t=mm.group(1) or mm.group(2)
        if t in labels and labels[t]<i:
            seg=body[labels[t]:i+1]
            ins=[x.split()[0] for x in seg if x.strip() and not x.strip().startswith(';') and not x.strip().startswith('.') and not x.strip().endswith(':')]
            v=sum(1 for x in ins if x.startswith('v_'))
            f=sum(1 for x in ins if re.match(r'v_(fma|fmac|mul|add|rcp)_f64',x))
            d=sum(1 for x in ins if 'dpp' in x)
            ds=sum(1 for x in ins if x.startswith('ds_'))
            print(f"loop {t} lines {labels[t]}-{i}: valu {v} f64 {f} dpp {d} ds {ds} total {len(ins)}")
