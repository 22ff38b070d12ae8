"""ORACLE -- CPU restatement of the device synthetic-data generator (TEST INFRASTRUCTURE).

Checker for sgvamp-py_amd/csrc/synth.hip.  Same recipe as the reference's
simulation (simulation/sim_gen_phen_mult.py:36-55), with the build's
counter-based RNG so genotypes are reproducible bit for bit on CPU and GPU:

  key = seed*0xD1B54A32D192ED03 + gmarker*0x9E3779B97F4A7C15 + n   (mod 2^64)
  h   = splitmix64(key);  x = [hi32(h) < T] + [lo32(h) < T],  T = floor(0.4*2^32)
  mean = S1/N,  std = sqrt((N*S2 - S1^2) / N^2)      (integer moments, exact)
  X_std = (x - mean)/std;  G = X_std/sqrt(N)          (sim_gen_phen_mult.py:40,53)
  R_b = G_b G_b^T (:55);  g = X_std^T beta (:44);  r_b = G_b y (:54)

Parity: genotypes/mean/std/G are bit-exact by construction; R and r differ from
the device only by summation order.  The reference's own simulation uses the
unseeded global RNG and has no fixtures, so this generator is "parity
unpinned" against the reference (it is checked against the HIP generator).
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def genotypes(seed, gm0, n, nsamp):
    """(n, nsamp) int array of Binomial(2, 0.4) draws for global markers gm0..gm0+n."""
    with np.errstate(over="ignore"):
        gi = (np.arange(n, dtype=np.uint64) + np.uint64(gm0))[:, None]
        ns = np.arange(nsamp, dtype=np.uint64)[None, :]
        key = (np.uint64(seed) * np.uint64(0xD1B54A32D192ED03)
               + gi * np.uint64(0x9E3779B97F4A7C15) + ns)
        h = splitmix64(key)
    T = np.uint64(1717986918)
    return ((h >> np.uint64(32)) < T).astype(np.int64) + ((h & np.uint64(0xFFFFFFFF)) < T).astype(np.int64)


def standardise(x):
    N = x.shape[1]
    S1 = x.sum(axis=1)
    S2 = (x * x).sum(axis=1)
    num = N * S2 - S1 * S1
    mean = S1.astype(np.float64) / float(N)
    sd = np.sqrt(num.astype(np.float64) / (float(N) * float(N)))
    Xs = (x.astype(np.float64) - mean[:, None]) / sd[:, None]
    return Xs, Xs / np.sqrt(float(N))


def block_data(seed, gm0, n, nsamp):
    x = genotypes(seed, gm0, n, nsamp)
    Xs, G = standardise(x)
    return Xs, G


def synth_problem(block_sizes, nsamp, beta, geno_seed, noise):
    """Full CPU generation: returns (R_blocks, r, g) for one cohort.
    noise: (nsamp,) phenotype noise w; y = g + w."""
    offs = np.concatenate([[0], np.cumsum(block_sizes)])
    Rb, gb = [], []
    for b, n in enumerate(block_sizes):
        Xs, G = block_data(geno_seed, offs[b], n, nsamp)
        Rb.append(G @ G.T)
        gb.append(Xs.T @ beta[offs[b]:offs[b + 1]])
    g = np.zeros(nsamp)
    for v in gb:
        g = g + v
    y = g + noise
    r = np.concatenate([block_data(geno_seed, offs[b], n, nsamp)[1] @ y
                        for b, n in enumerate(block_sizes)])
    return Rb, r, g, gb
