import re,collections,sys
# usage: loopstat.py file.s kernel_substring  -> opcode mix of every loop (by back-edge ranges) and totals
s=open(sys.argv[1]).read().split('\n')
i=[k for k,l in enumerate(s) if re.match(r'^_Z\w*%s\w*:'%sys.argv[2],l)][0]
body=[]
for l in s[i+1:]:
    if l.startswith('.Lfunc_end'): break
    body.append(l)
labels={l.split(':')[0]:k for k,l in enumerate(body) if re.match(r'^\.LBB\w+:',l)}
loops=[]
for k,l in enumerate(body):
    m=re.search(r's_(?:c)?branch\w*\s+(\.LBB\w+)',l)
    if m and m.group(1) in labels and labels[m.group(1)]<k:
        loops.append((labels[m.group(1)],k))
def mix(lines):
    return collections.Counter(l.strip().split()[0] for l in lines if l.strip() and not l.strip().startswith(';') and not l.strip().startswith('.') and not l.strip().endswith(':'))
tot=mix(body)
print('total', sum(tot.values()), 'valu', sum(v for k,v in tot.items() if k.startswith('v_')))
for a,b in loops:
    o=mix(body[a:b+1])
    print('loop', a, b, 'instr', sum(o.values()), 'valu', sum(v for k,v in o.items() if k.startswith('v_')), 'mac', o['v_mad_u64_u32'])
    if len(sys.argv)>3: 
        for k,v in o.most_common(int(sys.argv[3])): print('   ',k,v)
txt='\n'.join(s)
m=re.search(r'\.name:\s+_Z\d+\w*%s\w*\s.*?\.private_segment_fixed_size:\s+(\d+).*?\.sgpr_count:\s+(\d+).*?\.vgpr_count:\s+(\d+)'%sys.argv[2], txt, re.S); print('scratch/sgpr/vgpr', m.groups())
