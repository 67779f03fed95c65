import itertools
# lanes of ds_read_b128 groups (guide): lane -> (row=lane&15, chunk=lane>>4)
groups = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
groups += [[l+32 for l in g] for g in groups]
def ok(key, rowbytes):
    # reads: bank slot (16B) mod 16 distinct within each group, for K-half m=0,1
    for m in (0,1):
        for g in groups:
            slots = set()
            for l in g:
                r, c = l & 15, (l >> 4) + 4*m
                addr = r*rowbytes + ((c ^ key[r]) << 4)
                slots.add((addr // 16) % 16)
            if len(slots) != 16: return False
    return True
def store_conf(key, rowbytes):
    worst = 0
    for nt in range(4):
        for k in (0,1):
            for half in (0,1):
                banks = {}
                for lane in range(32*half, 32*half+32):
                    kq, j = lane >> 4, lane & 15
                    co = nt*16 + j
                    r = kq*4 + 2*k + (co & 1)
                    c = co >> 3
                    addr = r*rowbytes + ((c ^ key[r]) << 4) + ((co & 7) >> 1)*4
                    b = (addr // 4) % 32
                    banks.setdefault(b, set()).add(addr)
                worst = max(worst, max(len(v) for v in banks.values()))
    return worst
best = None
for M in itertools.product(range(8), repeat=4):  # key = xor of M[i] for set bits i of row
    key = []
    for r in range(16):
        v = 0
        for i in range(4):
            if r >> i & 1: v ^= M[i]
        key.append(v)
    if ok(key, 128):
        sc = store_conf(key, 128)
        if best is None or sc < best[0]: best = (sc, M, key)
print(best)
