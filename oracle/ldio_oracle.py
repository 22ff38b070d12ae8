"""ORACLE -- loop restatement of the reference's PLINK .ld exchange (TEST INFRASTRUCTURE).

src/main.py:203-257, all cohort ranks in one process: cohort k requests from
cohort j the markers whose source is j (source as src/main.py:151-162
computes it, passed in), j answers with every entry of its own table touching
a requested marker -- scanning its whole table once per requested marker, in
the reference's loop order -- and with its r at those markers.  Checker for
the vectorised loader sgvamp-py_amd/ldio.py:load_plink_ld_all
(tests/test_cli_io.py); never imported by the product path.
"""
import numpy as np


def exchange(own, sources, r, M):
    """own[k] = (indA, indB, R) lists of cohort k's table (reference-indexed);
    sources[k] (M,) = the cohort k asks for each marker.  Returns the per-cohort
    (ind_r, ind_c, v) COO triplets of R = I + pairs + transposed pairs
    (main.py:251-257) and the updated r (K, M)."""
    K = len(own)
    r_in = np.asarray(r, dtype=np.float64)
    r_out = r_in.copy()
    out = []
    for k in range(K):
        indA, indB, R_col = list(own[k][0]), list(own[k][1]), list(own[k][2])
        source = sources[k]
        for j in range(K):                                   # main.py:209-225, 228-246
            if j == k or j not in source:
                continue
            req = [i for i in range(M) if source[i] == j]
            jA, jB, jC = own[j]
            for ind in req:
                for i, corr in enumerate(jC):
                    if jA[i] == ind or jB[i] == ind:
                        indA.append(jA[i])
                        indB.append(jB[i])
                        R_col.append(corr)
            r_out[k][source == j] = r_in[j][req]
        ind_r = list(range(M)) + indA + indB                  # main.py:251-257
        ind_c = list(range(M)) + indB + indA
        v = list(np.ones(M)) + R_col + R_col
        out.append((ind_r, ind_c, v))
    return out, r_out
