"""LDS bank model of the attention V^T staging (ds_write_b32 stores, 32-lane groups, bank (a/4) mod 32) and its
fragment reads (ds_read_b128, 16-lane groups, bank (a/4) mod 64; MI355X_MICROARCH.md LDS table): worst-case ways per
instruction for the original layout and the best per-column-chunk XOR swizzle of the 16-byte chunk index.
usage: python tools/attn_banks.py"""
import itertools
VST2=68  # dwords per V^T row
def pos_of(row):  # forward's permuted position of key `row` (even) within its 16-group
    kk=row&15
    return (row&~15)+8*((kk>>2)&1)+(((kk>>3)<<2)|(kk&3))
def write_conf(D, s, mapping):
    CH=D//4; worst=0; tot=0; cnt=0
    items=[(e//CH, e%CH) for e in range(64*CH)] if mapping=='chfast' else [(e%64, e//64) for e in range(64*CH)]
    for w0 in range(0, len(items), 32):
        grp=items[w0:w0+32]
        for j in range(4):  # the 4 dword stores vt[0], vt[VST/2], vt[VST], vt[3VST/2]
            banks={}
            for kp,ch in grp:
                row=4*ch+j
                p=pos_of(2*kp)
                c16=p//8; c16s=c16 ^ s(ch)
                dw=row*VST2 + (c16s*8 + p%8)//2
                banks.setdefault(dw%32,set()).add(dw)
            m=max(len(v) for v in banks.values()); worst=max(worst,m); tot+=m; cnt+=1
    return worst, tot/cnt
def read_conf(D, s):
    groups=[[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
    worst=0
    for c16 in range(16):
        for g in groups:
            banks={}
            for l in g:
                dd=l
                if dd>=D: continue
                ch=dd>>2
                dw=dd*VST2 + 4*(c16 ^ s(ch))
                for q in range(4):
                    banks.setdefault((dw+q)%64,set()).add(dw+q)
            m=max(len(v) for v in banks.values()); worst=max(worst,m)
    return worst
for D in (16,24,32):
    print("D",D,"orig write",write_conf(D,lambda ch:0,'chfast'),"read",read_conf(D,lambda ch:0))
    best=None
    for tab in itertools.product(range(4),repeat=D//4):
        s=lambda ch,t=tab: t[ch]*1
        w=write_conf(D,s,'chfast'); r=read_conf(D,s)
        key=(w[0],w[1],r)
        if best is None or key<best[0]: best=(key,tab)
    print("  best swizzle table", best)
