#!/usr/bin/env python3
"""Attribute the VALU / MFMA / LDS instructions of a loop in a hipcc -S -g assembly file to source
lines through its .loc directives.  Usage: isa_line_attrib.py file.s first_line last_line [top]
(used for profiles/r06/c5_valu_attribution.txt: the C5 kernel compiled with -g, its step loop)."""
import re,collections,sys
L=open(sys.argv[1]).read().split('\n')
s,e=int(sys.argv[2]),int(sys.argv[3])
files={}
for l in L:
    m=re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"',l)
    if m: files[int(m.group(1))]=m.group(2)
cur=None
byline=collections.Counter(); byfile=collections.Counter(); mf=collections.Counter(); lds=collections.Counter()
for i in range(s,e):
    t=L[i].strip()
    m=re.match(r'\.loc\s+(\d+)\s+(\d+)',t)
    if m: cur=(files.get(int(m.group(1))),int(m.group(2))); continue
    if t.startswith('v_'):
        if 'mfma' in t: mf[cur]+=1; continue
        byline[cur]+=1; byfile[cur[0] if cur else None]+=1
    if t.startswith('ds_'): lds[cur[0] if cur else None]+=1
tot=sum(byline.values())
print('VALU static in loop',tot,'mfma',sum(mf.values()),'lds',dict(lds))
for k,v in byfile.most_common(): print('%5d %5.1f%% %s'%(v,100*v/tot,k))
print()
for k,v in byline.most_common(int(sys.argv[4]) if len(sys.argv)>4 else 30): print('%5d %s'%(v,k))
