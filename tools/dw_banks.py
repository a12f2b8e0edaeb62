"""gfx950 LDS bank model of the large-batch weight-gradient kernel's image
(iwae_dwgrad.hip, cdna_hip_programming.md T10 layout (b)): worst-case ways of
its ds_read_b64_tr_b16 fragment reads (64 banks per 32-lane half) and of its
row-major ds_write_b64 staging writes (32 banks per 16-lane group)."""
def swz(k): return ((k & 3) << 2) | ((k >> 2) & 3)
def off(k, cb, ch):            # bytes: col block cb (128 bf16 = 256 B rows, 32 rows), chunk ch of 16 B
    return cb * 8192 + 256 * k + 16 * (ch ^ swz(k))
worst = 0
# transposed reads: tile t (16 cols), h in {0,1}; lane l: group g = l>>4, i = l & 15 -> q = i >> 2, p = i & 3
for t in range(16):
    cb, c0 = (16 * t) >> 7, (16 * t) & 127
    for h in range(2):
        addrs = []
        for l in range(64):
            g, i = l >> 4, l & 15
            q, p = i >> 2, i & 3
            r0 = 8 * g + 4 * h
            addrs.append(off(r0 + q, cb, (c0 >> 3) + (p >> 1)) + 8 * (p & 1))
        for half in range(2):
            banks = {}
            for a in addrs[32 * half:32 * half + 32]:
                for d in range(2):
                    b = (a // 4 + d) % 64
                    banks[b] = banks.get(b, 0) + 1
            worst = max(worst, max(banks.values()))
print("tr read worst way", worst)
# writes: ds_write_b64, 16 contiguous lanes per group, bank (a/4) mod 32; lanes = consecutive quads of one row
worst = 0
for nq in (16, 32, 64):
    for row in range(32):
        for g0 in range(0, nq, 16):
            banks = {}
            for l in range(16):
                cq = g0 + l
                c = 4 * cq
                a = off(row, c >> 7, (c & 127) >> 3) + 2 * (c & 7)
                for d in range(2):
                    b = (a // 4 + d) % 32
                    banks[b] = banks.get(b, 0) + 1
            worst = max(worst, max(banks.values()))
print("write worst way", worst)
