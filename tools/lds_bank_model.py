"""Host model of LDS bank groups for the NTT's 1024-point / 4-line tile (csrc/kernels.hip Lds<10, 4096>).

A 16-byte element spans 4 of the 64 banks, so a 16-lane quarter-wave of ds_read/write_b128 is conflict-free
when its slots differ in the low 4 bits.  For every phase of the kernels that use the tile -- the pass-1/2
load order (rotated, bit-reversed), the stores, the single-pass load, and each radix-4 round with either the
library's thread-to-butterfly mapping or the wave-uniform-twiddle mapping of rounds h <= 16 -- prints the
worst multiplicity over all quarter-waves (1 = conflict-free) for the round-1 swizzle and the current one.
Usage: python3 tools/lds_bank_model.py
"""
# host model of LDS bank groups (slot & 15) per quarter-wave for every phase of a 1024-point / 4-line tile
def bitrev(x, b):
    return int(format(x, f'0{b}b')[::-1], 2)
def make(sw):
    def idx(line, pos): return line * 1024 + (sw(pos) ^ ((line & 3) << 2))
    return idx
def worst(acc):  # acc: list of 64 slots (a wave); returns max multiplicity over quarter-waves
    w = 1
    for qw in range(4):
        s = [x & 15 for x in acc[16 * qw:16 * qw + 16]]
        w = max(w, max(s.count(v) for v in set(s)))
    return w
def phases(idx, remap):
    out = {}
    # load
    m = 1
    for it in range(4):
        for wv in range(16):
            acc = []
            for l in range(64):
                e = it * 1024 + wv * 64 + l
                line, v = e % 4, e // 4
                k1 = ((v & 3) << 8) | (v >> 2)
                acc.append(idx(line, bitrev(k1, 10)))
            m = max(m, worst(acc))
    out['load'] = m
    m = 1
    for it in range(4):
        for wv in range(16):
            acc = [idx((it * 1024 + wv * 64 + l) % 4, (it * 1024 + wv * 64 + l) // 4) for l in range(64)]
            m = max(m, worst(acc))
    out['store'] = m
    for LG in (1, 3, 5, 7, 9):
        h = 1 << (LG - 1); LH = LG - 1
        m = 1
        for wv in range(16):
            for k in range(4):
                acc = []
                for l in range(64):
                    if remap and h <= 16:
                        j = wv >> (4 - LH); pidx = ((wv & ((16 >> LH) - 1)) << 6) | l
                        line = pidx >> (8 - LH); grp = pidx & ((256 >> LH) - 1)
                    else:
                        q = wv * 64 + l; line = q >> 8; local = q & 255; j = local & (h - 1); grp = local >> LH
                    acc.append(idx(line, grp * 4 * h + j + k * h))
                m = max(m, worst(acc))
        out[f'h={h}'] = m
    return out
old = lambda x: x ^ (((x >> 4) & 3) * 5)
new = lambda x: x ^ ((x >> 4) & 15) ^ ((x >> 8) & 3)
print('round-1 swizzle, library mapping :', phases(make(old), False))
print('round-1 swizzle, uniform h<=16   :', phases(make(old), True))
print('current swizzle, uniform h<=16   :', phases(make(new), True))
def extra(idx):
    out = {}
    m = 1
    for it in range(4):
        for wv in range(16):
            acc = []
            for l in range(64):
                e = it * 1024 + wv * 64 + l
                acc.append(idx(e >> 10, bitrev(e & 1023, 10)))
            m = max(m, worst(acc))
    out['single_load'] = m
    m = 1
    for it in range(4):
        for wv in range(16):
            acc = [idx((it * 1024 + wv * 64 + l) >> 10, (it * 1024 + wv * 64 + l) & 1023) for l in range(64)]
            m = max(m, worst(acc))
    out['pass1/single store'] = m
    return out
print('current swizzle, other phases   :', extra(make(new)), ' round-1 swizzle:', extra(make(old)))

# the 4096-point / 1-line tile (2^22 pass 1, single-pass n = 4096)
def check12(sw, LOGM=12):
    M = 1 << LOGM; idx = lambda pos: sw(pos)
    out = {}
    R = 4
    m = 1
    for it in range(4):
        for wv in range(16):
            acc = []
            for l in range(64):
                v = it * 1024 + wv * 64 + l
                k = ((v & 15) << (LOGM - R)) | (v >> R)
                acc.append(idx(bitrev(k, LOGM)))
            m = max(m, worst(acc))
    out['load'] = m
    m = 1
    for it in range(4):
        for wv in range(16):
            m = max(m, worst([idx(it * 1024 + wv * 64 + l) for l in range(64)]))
    out['store'] = m
    m = 1
    for it in range(4):
        for wv in range(16):
            m = max(m, worst([idx(bitrev(it * 1024 + wv * 64 + l, LOGM)) for l in range(64)]))
    out['single_load'] = m
    for LG in range(1, LOGM, 2):
        h = 1 << (LG - 1); LH = LG - 1
        for uni in ((False, True) if h <= 16 else (False,)):
            m = 1
            for wv in range(16):
                for k in range(4):
                    acc = []
                    for l in range(64):
                        if uni:
                            j = wv >> (4 - LH); pidx = ((wv & ((16 >> LH) - 1)) << 6) | l; grp = pidx
                        else:
                            q = wv * 64 + l; j = q & (h - 1); grp = q >> LH
                        acc.append(idx(grp * 4 * h + j + k * h))
                    m = max(m, worst(acc))
            out[f'h={h}{" uni" if uni else ""}'] = m
    return out
new12 = lambda x: x ^ ((x >> 4) & 15) ^ ((x >> 8) & 3) ^ (((x >> 10) & 3) << 2)
print('LOGM 12 round-1 swizzle      :', check12(old))
print('LOGM 12 current swizzle      :', check12(new12))


# ---- round 5 experiment (measured, removed: DESIGN.md §4 dead ends, profiles/r05b_ab_wave_local_ntt.txt): a tile
# layout for wave-local NTT rounds (one block barrier per pass-2 tile instead of four) and the lane maps of its phases
def wl_idx(line, pos):
    f = (((pos >> 4) ^ (pos >> 6) ^ (pos >> 8)) & 3) << 2
    return (line << 10) | (pos ^ line ^ f)


def wl_phases():
    out = {}
    def run(name, lanes):  # lanes(w, l) -> list of (line, pos) the lane touches, one per access
        m = 1
        for w in range(16):
            per = [lanes(w, l) for l in range(64)]
            for k in range(len(per[0])):
                m = max(m, worst([wl_idx(*per[l][k]) for l in range(64)]))
        out[name] = m
    # round 1 (first_round_from's lane order: line = q % 4, g = q / 4; positions 4g .. 4g+3)
    run('r1 write (A)', lambda w, l: [(l & 3, 4 * ((w << 4) | (l >> 2)) + t) for t in range(4)])
    # round 2 (A): j = quarter, line = l & 3, grp = (w << 2) | bits 4-5
    run('r2 (A)', lambda w, l: [(l & 3, ((w << 2) | ((l >> 2) & 3)) * 16 + (l >> 4) + 4 * t) for t in range(4)])
    # round 3 (B): j = w, line = l & 3, grp = l >> 2 (bits 6-9)
    run('r3 (B)', lambda w, l: [(l & 3, (l >> 2) * 64 + w + 16 * t) for t in range(4)])
    # round 4 (B): j = w | bits 4-5 from the quarter, grp = bits 8-9
    run('r4 (B)', lambda w, l: [(l & 3, ((l >> 2) & 3) * 256 + (w | (((l >> 4) & 3) << 4)) + 64 * t) for t in range(4)])
    # round 5, pass 2 (B): j = w | (l >> 2) << 4
    run('r5 pass 2 (B)', lambda w, l: [(l & 3, (w | ((l >> 2) << 4)) + 256 * t) for t in range(4)])
    # round 5, pass 1 (C): line = l >> 4, j = (w << 4) | (l & 15)
    run('r5 pass 1 (C)', lambda w, l: [(l >> 4, ((w << 4) | (l & 15)) + 256 * t) for t in range(4)])
    return out


print('wave-local tile (round-5 experiment)   :', wl_phases())
