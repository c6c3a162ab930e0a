"""LDS bank-conflict model of k_resnet_h2's activation image (design check, CPU only).

Model (MI355X_MICROARCH.md §LDS): a ds_read_b128 is serviced in four 16-lane groups
{0-3,12-15,20-27}, {4-11,16-19,28-31} (+32); a group costs one LDS cycle per distinct address on
its busiest bank (bank = (byte address / 4) mod 64). A ds_write_b64 is four groups of 16
contiguous lanes, banks (a / 4) mod 32.

Image (csrc/rvz_resnet.hip CfgH): per k-step plane, rows of 32 halves (4 16-byte slots), slot q
of row r at q ^ ((r >> 1) & 3); off-board taps read zero row ZROW + (r & 7).
B operand of v_mfma_f32_16x16x32_f16: lane l reads pixel tile*16 + (l & 15), slot l >> 4.
Epilogue: lane l writes channels 4 (l >> 4) .. +3 of pixel tile*16 + (l & 15) (8 bytes).

    python tools/lds_banks.py        # LDS cycles per read / b64 write / b128 write (ideal 4 / 4 / 8)
"""
READ_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
READ_GROUPS += [[lane + 32 for lane in g] for g in READ_GROUPS]


def group_cycles(addrs, groups, width, nbanks):
    tot = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for b in range(width // 4):
                banks.setdefault((a // 4 + b) % nbanks, set()).add(a)
        tot += max(len(v) for v in banks.values())
    return tot


def at(row, q, swz):
    return (row * 32 + 8 * (q ^ swz(row))) * 2          # bytes within a k-step plane


def read_cycles(nboard, bs, swz, zero_rows=8):
    zrow, tot, n = nboard * 64, 0, 0
    for pt in range(nboard * 4):
        for t in range(9):
            addrs = {}
            for lane in range(64):
                px = pt * 16 + (lane & 15)
                r, c = (px & 63) >> 3, px & 7
                dr, dc = t // 3 - 1, t % 3 - 1
                nat = px + dr * 8 + dc
                ok = 0 <= r + dr < bs and 0 <= c + dc < bs
                row = nat if ok else zrow + (nat & (zero_rows - 1))
                addrs[lane] = at(row, lane >> 4, swz)
            tot += group_cycles(addrs, READ_GROUPS, 16, 64)
            n += 1
    return tot / n


def write_cycles(nboard, swz):
    groups = [list(range(g, g + 16)) for g in range(0, 64, 16)]
    tot, n = 0, 0
    for pt in range(nboard * 4):
        for ct in range(2):                              # channel tiles within a k-step plane
            addrs = {}
            for lane in range(64):
                px = pt * 16 + (lane & 15)
                n0 = ct * 16 + 4 * (lane >> 4)
                addrs[lane] = at(px, n0 >> 3, swz) + (n0 & 4) * 2
            tot += group_cycles(addrs, groups, 8, 32)
            n += 1
    return tot / n


def write128_cycles(nboard, swz):
    """RVZ_H2_W128: after v_permlane16_swap, lane quad q writes 8 channels (16 B) of part q & 1,
    channels 8 (q >> 1) .. +7 of its channel tile, at pixel tile*16 + (lane & 15); ds_write_b128
    is serviced in 8 groups of 8 contiguous lanes, banks (a / 4) mod 32. The two parts are planes
    PLANE halves apart (a multiple of 16 B; the part-1 plane is placed arbitrarily here: lanes of
    one group never mix parts)."""
    groups = [list(range(g, g + 8)) for g in range(0, 64, 8)]
    plane = (nboard * 64 + 8) * 32 * 2                   # bytes of one part's k-step planes (KS=1)
    tot, n = 0, 0
    for pt in range(nboard * 4):
        for ct in range(2):
            addrs = {}
            for lane in range(64):
                q = lane >> 4
                px = pt * 16 + (lane & 15)
                n8 = ct * 16 + 8 * (q >> 1)
                addrs[lane] = at(px, n8 >> 3, swz) + (q & 1) * plane
            tot += group_cycles(addrs, groups, 16, 32)
            n += 1
    return tot / n


def main():
    cur = lambda r: (r >> 1) & 3                        # noqa: E731
    first = lambda r: (r >> 1) & 2                      # noqa: E731  (the first h2 version)
    for name, swz, zr in (("(r>>1)&3, 8 zero rows", cur, 8), ("(r>>1)&2, 1 zero row", first, 1)):
        for nb, bs in ((2, 8), (2, 6), (1, 8), (1, 6)):
            print(f"{name:24s} NB={nb} {bs}x{bs}: read {read_cycles(nb, bs, swz, zr):.2f} "
                  f"write b64 {write_cycles(nb, swz):.2f} (ideal 4) write b128 "
                  f"{write128_cycles(nb, swz):.2f} (ideal 8) LDS cycles")


if __name__ == "__main__":
    main()
