"""Lane-level NumPy restatement of k_als_wave (csrc/mf_als.hip) for ONE entity.

Test infrastructure: it models the kernel's data layout and step order (the
MFMA tile layout of the Gramian, the pivot-row publish with its masks and
double buffer, the row-per-lane right-hand columns, the register back
substitution over transposed diagonal tiles) in float64, so that a layout
or masking mistake shows up as a wrong solution on the CPU, before a GPU
run.  It is not an oracle for the GPU results (oracle.als_half_sweep is).

Lane L = c + 32 h of the 64-lane wave; tile (I, J), register i holds the
Gramian element (32 I + ra(i, h), 32 J + c), ra(i, h) = (i & 3) + 8 (i >> 2)
+ 4 h (the v_mfma_f32_32x32x2_f32 accumulator layout).
"""

import numpy as np

LANES = np.arange(64)
C = LANES & 31
H = LANES >> 5


def ra(i, h):
    return (i & 3) + 8 * (i >> 2) + 4 * h


def solve(nt, k, Z, t, reg):
    """x = [w; b] of (Y^T Y + reg I) x = Y^T t, Y = [Z, 1], as k_als_wave<nt>."""
    kp = 32 * nt
    cnt = Z.shape[0]
    tiles = [(I, J) for J in range(nt) for I in range(J + 1)]
    q = {tj: n for n, tj in enumerate(tiles)}
    Zp = np.zeros((cnt, kp))
    Zp[:, :k] = Z
    # 1. Gramian tiles and the right-hand columns (both halves summed)
    m = np.zeros((len(tiles), 16, 64))
    for (I, J), n in q.items():
        for i in range(16):
            m[n, i] = (Zp[:, 32 * I + ra(i, H)] * Zp[:, 32 * J + C]).sum(0)
    fz = np.array([(t[:, None] * Zp[:, 32 * I + C]).sum(0) for I in range(nt)])
    sz = np.array([Zp[:, 32 * I + C].sum(0) for I in range(nt)])
    gsum = t.sum()
    nr = (kp + 63) // 64
    fr = np.zeros((nr, 64))
    sr = np.zeros((nr, 64))
    for x in range(nr):
        for I in range(2 * x, min(2 * x + 2, nt)):
            sel = (I & 1) == H
            fr[x][sel] = fz[I][sel]
            sr[x][sel] = sz[I][sel]
        fr[x][LANES + 64 * x >= kp] = 0.0
        sr[x][LANES + 64 * x >= kp] = 0.0
    for I in range(nt):
        n = q[(I, I)]
        for i in range(16):
            dg = np.where(32 * I + C < k, m[n, i] + reg, 1.0)
            m[n, i] = np.where(ra(i, H) == C, dg, m[n, i])
    # 2. elimination: publish row j, rank-1 update, f / s row-per-lane
    prow = np.zeros((2, kp))
    dreg = np.ones((nr, 64))
    st = {}

    def publish(Ij, j):
        jl = j - 32 * Ij
        ij = (jl & 3) | ((jl >> 3) << 2)
        hj = (jl >> 2) & 1
        u = np.zeros((nt, 64))
        dv = None
        for J in range(Ij, nt):
            v = m[q[(Ij, J)], ij]
            uv = v[C + 32 * hj]                        # permlane32_swap, half hj
            b = 32 * J + C
            u[J] = np.where(b > j, uv, 0.0)
            prow[j & 1][b[:32]] = u[J][:32]
            if J == Ij:
                dv = uv
        st["u"], st["d"] = u, dv[jl]
        st["r"] = 1.0 / st["d"]

    for Ij in range(nt):
        publish(Ij, 32 * Ij)
        for jl in range(32):
            j = 32 * Ij + jl
            pr = prow[j & 1].copy()
            u, r, d = st["u"], st["r"], st["d"]
            w = np.array([np.zeros(64) if J < Ij else u[J] * -r for J in range(nt)])
            fjr = fr[Ij >> 1][j & 63] * -r
            sjr = sr[Ij >> 1][j & 63] * -r
            dreg[Ij >> 1] = np.where(LANES == (j & 63), d, dreg[Ij >> 1])

            def update_row(I):
                lmul = np.array([pr[32 * I + ra(i, H)] for i in range(16)])
                for J in range(I, nt):
                    m[q[(I, J)]] += lmul * w[J]

            update_row(Ij)
            if jl < 31:
                publish(Ij, j + 1)
            for I in range(Ij + 1, nt):
                update_row(I)
            for x in range(nr):
                a = LANES + 64 * x
                la = np.where((a > j) & (a < kp), pr[np.minimum(a, kp - 1)], 0.0)
                fr[x] += la * fjr
                sr[x] += la * sjr
    # 3. border and back substitution from the tile registers
    dinv = 1.0 / dreg
    num = (sr * fr * dinv).sum()
    den = (sr * sr * dinv).sum()
    bias = (gsum - num) / ((cnt + reg) - den)
    y = fr - bias * sr
    xc = np.zeros((nt, 64))
    for I in range(nt - 1, -1, -1):
        src = 32 * (I & 1) + C
        yc = y[I >> 1][src]
        dc = dinv[I >> 1][src]
        off = np.zeros(64)
        if I < nt - 1:
            S = np.zeros((32, 33))
            for i in range(16):
                pv = sum(m[q[(I, J)], i] * xc[J] for J in range(I + 1, nt))
                S[ra(i, H), C] = pv
            sacc = np.array([S[C[l], 16 * H[l]:16 * H[l] + 16].sum() for l in range(64)])
            off = sacc + sacc[LANES ^ 32]
        rc = yc - off
        S = np.zeros((32, 33))
        for i in range(16):
            S[ra(i, H), C] = m[q[(I, I)], i]
        T = np.array([S[C, ra(i, H)] for i in range(16)])
        acc = np.zeros(64)
        xi = np.zeros(64)
        for tl in range(31, -1, -1):
            it = (tl & 3) + 4 * (tl >> 3)
            ht = (tl >> 2) & 1
            xv = ((rc - acc)[tl] - acc[32 + tl]) * dc[tl]
            xi = np.where(C == tl, xv, xi)
            acc = acc + np.where((H == ht) & (C < tl), T[it], 0.0) * xv
        xc[I] = xi
    w_out = np.concatenate([xc[I][:32] for I in range(nt)])[:k]
    return w_out, bias
