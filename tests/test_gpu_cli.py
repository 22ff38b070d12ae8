"""The process seam end to end on the GPU: sgvamp-py_amd/main.py with the
reference's flags and file formats (src/main.py:27-330).

* a golden case written out as the reference's input files (.npy LD, .npy r,
  .bim, true signal) -> the output .bin/.csv files match the reference's;
* PLINK .ld text LD (with a cohort missing markers) gives the same run as .npz
  files holding the matrices the .ld loader builds (loader semantics:
  tests/test_cli_io.py)."""
import os

import numpy as np
import pytest

from tests.golden import Case

pytestmark = pytest.mark.gpu


def _write_bim(path, names, coords):
    with open(path, "w") as f:
        for n, c in zip(names, coords):
            f.write("1\t%s\t0\t%d\tA\tG\n" % (n, c))


def _maxrel(a, b):
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-300))


def _flags(f):
    def j(v):
        return ",".join(repr(float(x)) for x in v)
    return ["--iterations", str(f["iterations"]), "--prior-vars", j(f["prior_vars"]),
            "--prior-probs", j(f["prior_probs"]), "--gamw", repr(float(f["gamw"])),
            "--gam1", repr(float(f["gam1"])), "--rho", repr(float(f["rho"])),
            "--cg-maxit", str(f["cg_maxit"]), "--em-prior-maxit", str(f["em_prior_maxit"]),
            "--learn-gamw", str(int(f["learn_gamw"])), "--lmmse-damp", str(int(f["lmmse_damp"])),
            "--s", repr(float(f["s"])), "--prior-update", f["prior_update"],
            "--update-prior-from", str(f["update_prior_from"]), "--seed", str(f["seed"])]


@pytest.mark.parametrize("name", ["k1_dense", "k1_mle"])
def test_cli_matches_reference_golden(name, tmp_path):
    import main

    c = Case(name)
    f = c.flags
    M = c.M
    R = np.zeros((M, M))
    o = 0
    for B in c.ld_blocks[0]:
        n = B.shape[0]
        R[o:o + n, o:o + n] = B
        o += n
    np.save(tmp_path / "R.npy", R)
    np.save(tmp_path / "r.npy", c.r[0])
    np.save(tmp_path / "beta.npy", c.beta)
    _write_bim(tmp_path / "c.bim", ["rs%d" % i for i in range(M)], range(1, M + 1))
    out = tmp_path / "out"
    out.mkdir()
    argv = ["--ld-files", str(tmp_path / "R.npy"), "--r-files", str(tmp_path / "r.npy"),
            "--true-signal-file", str(tmp_path / "beta.npy"), "--out-dir", str(out),
            "--out-name", name, "--N", str(c.N[0]), "--M", str(M), "--K", "1",
            "--bim-files", str(tmp_path / "c.bim")] + _flags(f)
    main.main(argv)
    for it in range(f["iterations"]):
        xb = np.fromfile(out / ("%s_xhat_it_%d.bin" % (name, it)))
        assert _maxrel(xb, c.xhat[it]) < 1e-8, it
    with open(out / ("%s_cohort_1.csv" % name)) as fh:
        rows = np.array([[float(x) for x in ln.split("\t")] for ln in fh.read().splitlines()[1:]])
    np.testing.assert_allclose(rows, c.cohort_csv[0], rtol=1e-5, atol=0)
    assert os.path.exists(out / (name + ".bim"))


def test_cli_plink_ld_equals_npz(tmp_path):
    import scipy.sparse

    import main
    from ldio import load_plink_ld_all, merge_bims

    rs = np.random.RandomState(4)
    M, nsamp = 240, 600
    names = ["rs%d" % i for i in range(M)]
    X = rs.normal(size=(nsamp, M))
    for b in range(0, M, 60):                      # 4 LD blocks of 60
        X[:, b + 1:b + 60] += 0.7 * X[:, b:b + 1]
    X = (X - X.mean(0)) / X.std(0) / np.sqrt(nsamp)
    C = X.T @ X
    beta = np.zeros(M)
    beta[rs.choice(M, 24, replace=False)] = rs.normal(0, np.sqrt(0.8 / 24), 24)
    missing = set(range(100, 115))                 # cohort 1 lacks 15 markers
    keep1 = [i for i in range(M) if i not in missing]
    cohorts = [list(range(M)), keep1]
    for k, idx in enumerate(cohorts):
        _write_bim(tmp_path / ("c%d.bim" % k), [names[i] for i in idx], [i + 1 for i in idx])
        with open(tmp_path / ("c%d.ld" % k), "w") as fh:
            fh.write(" CHR_A BP_A SNP_A CHR_B BP_B SNP_B R\n")
            for a in idx:
                for b in idx:
                    if a < b and a // 60 == b // 60:
                        fh.write(" 1 %d %s 1 %d %s %r\n" % (a + 1, names[a], b + 1, names[b],
                                                                   float(C[a, b])))
        y = X @ beta * np.sqrt(nsamp) + rs.normal(0, np.sqrt(0.2), nsamp)
        np.save(tmp_path / ("r%d.npy" % k), (X.T @ y)[idx])
    bims = [str(tmp_path / ("c%d.bim" % k)) for k in range(2)]
    common = ["--N", "600,600", "--M", "%d,%d" % (M, len(keep1)), "--K", "2",
              "--bim-files", ",".join(bims), "--iterations", "5", "--prior-vars",
              "0,%r" % (0.8 / 24 / 2), "--prior-probs", "0.9,0.1", "--seed", "3"]
    out_a = tmp_path / "a"
    out_a.mkdir()
    main.main(["--ld-files", ",".join(str(tmp_path / ("c%d.ld" % k)) for k in range(2)),
               "--r-files", ",".join(str(tmp_path / ("r%d.npy" % k)) for k in range(2)),
               "--out-dir", str(out_a), "--out-name", "a"] + common)
    # the same matrices and exchanged r vectors as .npz / reference-ordered .npy
    df, lists = merge_bims(bims)
    ref = list(df["Variant"])
    r_ref = np.zeros((2, M))
    for k, idx in enumerate(cohorts):
        r_ref[k][idx] = np.load(tmp_path / ("r%d.npy" % k))
    mats, r_x = load_plink_ld_all([str(tmp_path / ("c%d.ld" % k)) for k in range(2)], r_ref, ref,
                                  lists, [600, 600])
    assert mats[1][105, 105] == 1.0 and r_x[1][105] == r_ref[0][105]   # filled from cohort 0
    for k in range(2):
        scipy.sparse.save_npz(tmp_path / ("R%d.npz" % k), mats[k])
        np.save(tmp_path / ("rx%d.npy" % k), r_x[k])
    out_b = tmp_path / "b"
    out_b.mkdir()
    full = ["--N", "600,600", "--M", "%d,%d" % (M, M), "--K", "2", "--iterations", "5",
            "--prior-vars", "0,%r" % (0.8 / 24 / 2), "--prior-probs", "0.9,0.1", "--seed", "3"]
    main.main(["--ld-files", ",".join(str(tmp_path / ("R%d.npz" % k)) for k in range(2)),
               "--r-files", ",".join(str(tmp_path / ("rx%d.npy" % k)) for k in range(2)),
               "--out-dir", str(out_b), "--out-name", "a"] + full)
    for it in range(5):
        a = np.fromfile(out_a / ("a_xhat_it_%d.bin" % it))
        b = np.fromfile(out_b / ("a_xhat_it_%d.bin" % it))
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("launch", ["env", "mpirun", "gpus"])
def test_cli_two_ranks_bitwise_equal_one_rank(tmp_path, launch):
    """main.py as 2 ranks (LD blocks sharded; both ranks on device 0 with the
    host exchange, since RCCL refuses two ranks per device), launched three
    ways: RANK/WORLD_SIZE set per process ("env"), only Open MPI's variables --
    the reference's own `mpirun -np 2 python main.py` (src/main.py:16-18) --
    ("mpirun"), and `main.py --gpus 2` starting its ranks itself ("gpus").  Every
    output .bin file is bitwise the single-process one (ordered per-block
    reductions) and the per-cohort CSV is identical: one job, not two copies."""
    import socket
    import subprocess
    import sys

    import scipy.sparse

    import main

    rs = np.random.RandomState(11)
    M, nsamp = 360, 800
    X = rs.normal(size=(nsamp, M))
    for b in range(0, M, 90):                       # 4 LD blocks of 90
        X[:, b + 1:b + 90] += 0.6 * X[:, b:b + 1]
    X = (X - X.mean(0)) / X.std(0) / np.sqrt(nsamp)
    C = X.T @ X
    mask = np.zeros((M, M), dtype=bool)
    for b in range(0, M, 90):
        mask[b:b + 90, b:b + 90] = True
    scipy.sparse.save_npz(tmp_path / "R.npz", scipy.sparse.csr_matrix(np.where(mask, C, 0.0)))
    beta = np.zeros(M)
    beta[rs.choice(M, 36, replace=False)] = rs.normal(0, np.sqrt(0.8 / 36), 36)
    y = X @ beta * np.sqrt(nsamp) + rs.normal(0, np.sqrt(0.2), nsamp)
    np.save(tmp_path / "r.npy", X.T @ y)
    np.save(tmp_path / "beta.npy", beta)

    def argv(out):
        return ["--ld-files", str(tmp_path / "R.npz"), "--r-files", str(tmp_path / "r.npy"),
                "--true-signal-file", str(tmp_path / "beta.npy"), "--out-dir", str(out),
                "--out-name", "t", "--N", str(nsamp), "--M", str(M), "--K", "1",
                "--iterations", "6", "--prior-vars", "0,%r" % (0.8 / 36),
                "--prior-probs", "0.9,0.1", "--seed", "4", "--s", "0.02"]

    one = tmp_path / "one"
    one.mkdir()
    main.main(argv(one))
    two = tmp_path / "two"
    two.mkdir()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import main; main.main(sys.argv[1:])"
            % os.path.join(root, "sgvamp-py_amd"))
    base = {k: v for k, v in os.environ.items()
            if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    base["SGV_EXCHANGE"] = "host"
    procs = []
    if launch == "gpus":
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(root, "sgvamp-py_amd", "main.py")] + argv(two)
            + ["--gpus", "2", "--device", "0"], env=base, stdout=subprocess.PIPE,
            stderr=subprocess.STDOUT, text=True))
    for r in range(2 if launch != "gpus" else 0):
        if launch == "env":
            env = dict(base, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2",
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        else:
            env = dict(base, OMPI_COMM_WORLD_RANK=str(r), OMPI_COMM_WORLD_SIZE="2",
                       OMPI_COMM_WORLD_LOCAL_RANK=str(r), OMPI_COMM_WORLD_LOCAL_SIZE="2",
                       OMPI_MCA_ess_base_jobid="cli%d" % port, SGV_COMM_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", code] + argv(two) + ["--device", "0"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out[-3000:]
    bins = sorted(f for f in os.listdir(one) if f.endswith(".bin"))
    assert len(bins) == 12 and bins == sorted(f for f in os.listdir(two) if f.endswith(".bin"))
    for f in bins:
        assert (one / f).read_bytes() == (two / f).read_bytes(), f
    assert (one / "t_cohort_1.csv").read_text() == (two / "t_cohort_1.csv").read_text()


def test_cli_banded_npz_vs_oracle(tmp_path):
    """A windowed (banded, not block-diagonal) LD matrix as .npz -- one band over
    all 9,000 markers, bw = 500 -- through main.py: stored as a packed band on
    the device, never densified on the host; the output files equal the oracle
    running scipy's CSR mat-vec on the same matrix (the reference's operator)."""
    import scipy.sparse

    import main
    from oracle import vamp_oracle as vo

    M, bw, N = 9000, 500, 4000
    A = vo.banded_ld(M, bw, seed=31)
    scipy.sparse.save_npz(tmp_path / "R.npz", A)
    rs = np.random.RandomState(6)
    cm = M // 25
    beta = np.zeros(M)
    beta[rs.choice(M, cm, replace=False)] = rs.normal(0, np.sqrt(0.6 / cm), cm) * np.sqrt(N)
    r = A @ beta + rs.normal(size=M) * np.sqrt(0.4)
    np.save(tmp_path / "r.npy", r)
    out = tmp_path / "out"
    out.mkdir()
    its = 6
    pv, pp = [0.0, 0.6 / cm], [0.96, 0.04]
    main.main(["--ld-files", str(tmp_path / "R.npz"), "--r-files", str(tmp_path / "r.npy"),
               "--out-dir", str(out), "--out-name", "band", "--N", str(N), "--M", str(M),
               "--K", "1", "--iterations", str(its), "--prior-vars", "0,%r" % pv[1],
               "--prior-probs", "0.96,0.04", "--gamw", "2", "--seed", "5", "--s", "0.02",
               "--lmmse-damp", "1"])
    t = vo.infer([vo.CsrLD(A, s=0.02)], [0], [r], [float(N)], its, rho=0.5, gamw=2.0, gam1=1e-6,
                 prior_vars=pv, prior_probs=pp, seed=5, lmmse_damp=True,
                 reducer=vo.Reducer("blocked", bounds=np.array([0, M])), rs_recurrence=True)
    for it in range(its):
        xb = np.fromfile(out / ("band_xhat_it_%d.bin" % it))
        assert _maxrel(xb, np.asarray(t["xhat"][it]).ravel()) < 1e-8, it


def test_cli_one_chromosome_band_over_two_ranks(tmp_path):
    """One chromosome of windowed LD as one .npz (src/main.py:199-200): main.py
    cuts the band into coupled pieces (65,536 + 84,464 markers), and `--gpus 2`
    puts one piece on each rank (halo exchange of the corner sources, both
    ranks on device 0 with the host exchange) -- every output .bin file and the
    cohort / metrics CSVs bitwise the single-process run's."""
    import subprocess
    import sys

    import scipy.sparse

    import main
    from oracle import vamp_oracle as vo

    M, bw, N = 150_000, 500, 5000
    A = vo.banded_ld(M, bw, seed=12, taps=8)
    scipy.sparse.save_npz(tmp_path / "R.npz", A)
    rs = np.random.RandomState(8)
    cm = M // 40
    beta = np.zeros(M)
    beta[rs.choice(M, cm, replace=False)] = rs.normal(0, np.sqrt(0.5 / cm), cm)
    np.save(tmp_path / "r.npy", A @ (beta * np.sqrt(N)) + rs.normal(size=M))
    np.save(tmp_path / "beta.npy", beta)

    def argv(out):
        return ["--ld-files", str(tmp_path / "R.npz"), "--r-files", str(tmp_path / "r.npy"),
                "--true-signal-file", str(tmp_path / "beta.npy"), "--out-dir", str(out),
                "--out-name", "chr", "--N", str(N), "--M", str(M), "--K", "1",
                "--iterations", "4", "--prior-vars", "0,%r" % (0.5 / cm),
                "--prior-probs", "0.97,0.03", "--seed", "3"]

    one = tmp_path / "one"
    one.mkdir()
    main.main(argv(one))
    two = tmp_path / "two"
    two.mkdir()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["SGV_EXCHANGE"] = "host"
    p = subprocess.run([sys.executable, os.path.join(root, "sgvamp-py_amd", "main.py")] + argv(two)
                       + ["--gpus", "2", "--device", "0"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    files = sorted(f for f in os.listdir(one) if f.endswith((".bin", ".csv")))
    assert len([f for f in files if f.endswith(".bin")]) == 8
    assert files == sorted(f for f in os.listdir(two) if f.endswith((".bin", ".csv")))
    for f in files:
        assert (one / f).read_bytes() == (two / f).read_bytes(), f


def test_simulate_writes_cli_inputs(tmp_path):
    """simulate.py (simulation/sim_gen_phen_mult.py on the device): per cohort its
    own genotypes, block-diagonal LD as a manifest of block files, r, y, beta and
    .bim files; every LD block, r and y equal the CPU restatement of the
    generator; main.py then runs on the files, matching the oracle on them."""
    import json

    import main
    import simulate
    from oracle import synth_oracle as so
    from oracle import vamp_oracle as vo

    M, N, K, seed = 2500, 600, 2, 11
    sizes = [1000, 1000, 500]
    out = str(tmp_path / "sim")
    p = simulate.simulate(out, N, M, K=K, block_size=1000, seed=seed)
    beta = np.load(p["beta"]).ravel()
    assert np.count_nonzero(beta) == M // 2
    lds, rs = [], []
    for k in range(K):
        w = np.random.RandomState(seed + 1000 + k).normal(0.0, np.sqrt(0.2), N)
        Rb, r, g, _ = so.synth_problem(sizes, N, beta, seed + 1 + 7919 * k, w)
        man = json.load(open(p["ld"][k]))
        assert man["block_sizes"] == sizes
        blocks = [np.load(os.path.join(str(tmp_path), fn)) for fn in man["files"]]
        for B, Bref in zip(blocks, Rb):
            assert _maxrel(B, Bref) < 1e-12
        rk = np.load(p["r"][k]).ravel()
        assert _maxrel(rk, r) < 1e-12
        assert _maxrel(np.load(p["phen"][k]).ravel(), g + w) < 1e-12
        lds.append(vo.BlockLD(blocks))
        rs.append(rk)
    cm = M // 2
    o = tmp_path / "out"
    o.mkdir()
    its = 3
    main.main(["--ld-files", ",".join(p["ld"]), "--r-files", ",".join(p["r"]),
               "--bim-files", ",".join(p["bim"]), "--true-signal-file", p["beta"],
               "--out-dir", str(o), "--out-name", "sim", "--N", "%d,%d" % (N, N),
               "--M", "%d,%d" % (M, M), "--K", str(K), "--iterations", str(its),
               "--prior-vars", "0,%r" % (0.8 / cm), "--prior-probs", "0.5,0.5", "--seed", "3"])
    t = vo.infer(lds, [0, 1], rs, [float(N)] * K, its, rho=0.5, gamw=5.0, gam1=1e-6,
                 prior_vars=[0.0, 0.8 / cm], prior_probs=[0.5, 0.5], seed=3,
                 reducer=vo.Reducer("blocked", bounds=lds[0].bounds), rs_recurrence=True)
    for it in range(its):
        xb = np.fromfile(o / ("sim_xhat_it_%d.bin" % it))
        assert _maxrel(xb, np.asarray(t["xhat"][it]).ravel()) < 1e-8, it
