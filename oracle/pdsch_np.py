"""PDSCH resource-element map restated from 36.211 6.3.5 / 6.10.1.2 rules (TEST INFRASTRUCTURE).

Independent of the product's pointer-walking restatement of srsran_pdsch_cp (pdsch.c:136-220):
a RE (symbol l of slot s, PRB n, subcarrier k) carries PDSCH iff the PRB is granted, l is past
the control region (slot 0), k is not a CRS position of any cell port (k = off mod 3 for 2/4
ports, k = off mod 6 for 1 port, in the CRS symbols l = 0, nsymb - 3 and l = 1 for 4 ports), and the
PRB is not one of the 6 (7 for odd N_PRB) centre PRBs in the PSS/SSS/PBCH symbols of
subframes 0/5 (pdsch_cp_skip_symbol, pdsch.c:83-112) -- for odd N_PRB the outer halves of the
two edge PRBs of that block still carry PDSCH (pdsch.c:178-203)."""


def crs_symbol(l, nof_ports, nsymb=7):
    return l == 0 or l == nsymb - 3 or (l == 1 and nof_ports == 4)


def crs_offset(l, nof_ports, cell_id):
    if nof_ports == 1:
        return cell_id % 6 if l == 0 else (cell_id + 3) % 6
    return cell_id % 3


def skipped(nof_prb, fdd, sf_idx, s, l, n, nsymb=7):
    if nof_prb // 2 - 3 <= n < nof_prb // 2 + 3 + nof_prb % 2:
        if fdd:
            if s == 0 and sf_idx in (0, 5) and l >= nsymb - 2:
                return True
        else:
            if s == 1 and sf_idx in (0, 5) and l >= nsymb - 1:
                return True
            if s == 0 and sf_idx in (1, 6) and l == 2:
                return True
        if s == 1 and sf_idx == 0 and l < 4:
            return True
    return False


# 36.211 Table 4.2-2 (uplink-downlink configurations) and Table 4.2-1 (DwPTS / GP / UpPTS symbols of the
# special-subframe configurations, normal CP); srsRAN's tables: phy_common.c:98-106, 140-149
TDD_PATTERN = ("DSUUUDSUUU", "DSUUDDSUUD", "DSUDDDSUDD", "DSUUUDDDDD", "DSUUDDDDDD", "DSUDDDDDDD", "DSUUUDSUUD")
TDD_SS_SYMBOLS = ((3, 10, 1), (9, 4, 1), (10, 3, 1), (11, 2, 1), (12, 1, 1), (3, 9, 2), (9, 3, 2), (10, 2, 2),
                  (11, 1, 1), (6, 6, 2))


def tdd_type(sf_config, sf_idx):
    return TDD_PATTERN[sf_config][sf_idx]


def tdd_nof_symb_slot(sf_config, ss_config, sf_idx, cp=0):
    """PDSCH symbols per slot of a TDD subframe (the grant's nof_symb_slot): the DwPTS of a special subframe
    filled slot by slot, every symbol of a downlink subframe."""
    nsymb = 6 if cp else 7
    if tdd_type(sf_config, sf_idx) != "S":
        return (nsymb, nsymb)
    dw = TDD_SS_SYMBOLS[ss_config][0]
    return (dw, 0) if dw < nsymb else (nsymb, dw - nsymb)


def re_table(nof_prb, nof_ports, cell_id, prb_mask, lstart, sf_idx, fdd=True, cp=0, nsl=None):
    """List of (grid index, crs_symbol) in PDSCH order; prb_mask[s][n]; cp 1 = extended (6 symbols a
    slot, CRS in l = 0 and 3); nsl = the grant's symbols per slot (a TDD special subframe's DwPTS), the
    grid rows of slot 1 starting at nsl[0] as srsran_pdsch_cp lays them (pdsch.c:160)."""
    nsymb = 6 if cp else 7
    nsl = nsl or (nsymb, nsymb)
    out = []
    for s in range(2):
        for l in range(lstart if s == 0 else 0, nsl[s]):
            lp = l + nsl[0] * s
            crs = crs_symbol(l, nof_ports, nsymb)
            off = crs_offset(l, nof_ports, cell_id)
            period = 6 if nof_ports == 1 else 3
            for n in range(nof_prb):
                if not prb_mask[s][n]:
                    continue
                ks = range(12)
                if skipped(nof_prb, fdd, sf_idx, s, l, n, nsl[s]):
                    if nof_prb % 2 == 0:
                        continue
                    if n == nof_prb // 2 - 3:
                        ks = range(6)
                    elif n == nof_prb // 2 + 3:
                        ks = range(6, 12)
                    else:
                        continue
                for k in ks:
                    if crs and k % period == off % period:
                        continue
                    out.append(((lp * nof_prb + n) * 12 + k, crs))
    return out
