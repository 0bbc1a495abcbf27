"""Generate the golden vectors of tests/golden/ (SURVEY.md §8(c)).

Producer: oracle/arwmh_np.py, the literal float64 restatement of the
reference (arwmh.py:140-207 + numpyro cholesky_update), fed the build's
Philox noise.  The reference itself (JAX/NumPyro) is not importable here, so
these vectors pin the restatement that the C oracle and the HIP kernels are
checked against.  Fixtures hold inputs and expected outputs only.

  eight_schools.npz   4 chains x 1000 steps (run key (0, 0), chains 0-3,
                      W = 0 as collect_states_logscale), states at the
                      ns_logscale grid points <= 1000 (190 points) and the
                      accept decision of every step
  gaussian64.npz      8 chains x 100 steps of the d = 64 correlated Gaussian
                      (BASELINE config 2 target), states at 7 step counts
  cholupdate.npz      rank-one update known answers (d = 1, 3, 8, 26, 64)

  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))

import arwmh_np as lit  # noqa: E402


def packed(L):
    d = L.shape[0]
    return np.concatenate([L[j:, j] for j in range(d)])


def run(potential, d, z0, keys, steps, record, num_warmup=0):
    C = z0.shape[0]
    rec = {k: [] for k in ("i", "z", "pe", "loc", "scale", "lam", "macc", "as_change")}
    acc = np.zeros((C, steps), bool)
    states = []
    for c in range(C):
        z = z0[c].astype(np.float64)
        states.append(lit.ARWMHState(0, z, float(potential(z)), 0.0,
                                     lit.ARWMHAdaptState(z.copy(), np.eye(d), 0.0), 0.0, keys[c]))
    snaps = {t: [None] * C for t in record}
    for c in range(C):
        s = states[c]
        for t in range(steps):
            bits, ubits = lit.step_noise(keys[c], s.i, d)
            xi = lit.normal_from_bits(bits[0])
            u = float(lit.unif01_from_bits(ubits[0]))
            s, a, _ = lit.sample(s, potential, xi, u, num_warmup=num_warmup)
            acc[c, t] = a
            if t + 1 in snaps:
                snaps[t + 1][c] = s
    for t in record:
        ss = snaps[t]
        rec["i"].append([s.i for s in ss])
        rec["z"].append([s.z for s in ss])
        rec["pe"].append([s.potential_energy for s in ss])
        rec["loc"].append([s.adapt_state.loc for s in ss])
        rec["scale"].append([packed(s.adapt_state.scale) for s in ss])
        rec["lam"].append([s.adapt_state.log_step_size for s in ss])
        rec["macc"].append([s.mean_accept_prob for s in ss])
        rec["as_change"].append([s.as_change for s in ss])
    out = {k: np.asarray(v, np.int32 if k == "i" else np.float32) for k, v in rec.items()}
    out["accept"] = acc
    out["steps_recorded"] = np.asarray(record, np.int32)
    return out


def main():
    import posteriors as P
    key = np.array([0, 0], np.uint32)

    # eight schools (non-centred), posteriordb data, d = 10
    data = P.EIGHT_SCHOOLS_DATA
    y, sg = data["y"].astype(np.float64), data["sigma"].astype(np.float64)
    arr, _ = P.eight_schools.pack_fn(data)
    C, d = 4, 10
    keys = lit.chain_keys(key, 0, C)
    z0 = np.random.default_rng(0).uniform(-2, 2, size=(C, d)).astype(np.float32)
    grid = [int(n) for n in lit.ns_logscale(3) if n <= 1000]
    out = run(lambda z: lit.eight_schools_potential(z, y, sg), d, z0, keys, 1000, grid)
    np.savez_compressed(os.path.join(HERE, "eight_schools.npz"), model_data=arr.astype(np.float32), J=8,
                        run_key=key, chain_keys=keys, init_z=z0, num_warmup=0, **out)

    # d = 64 correlated Gaussian
    g = P.correlated_gaussian(64)
    gdata, _ = g.pack("cpu")
    gdata = gdata.numpy()
    m, Pm, c0 = gdata[:64].astype(np.float64), gdata[64:64 + 4096].reshape(64, 64).astype(np.float64), float(gdata[-1])
    C, d = 8, 64
    keys = lit.chain_keys(key, 0, C)
    z0 = np.random.default_rng(64).uniform(-2, 2, size=(C, d)).astype(np.float32)
    out = run(lambda z: lit.gaussian_potential(z, m, Pm, c0), d, z0, keys, 100, [1, 2, 5, 10, 20, 50, 100])
    np.savez_compressed(os.path.join(HERE, "gaussian64.npz"), model_data=gdata, run_key=key, chain_keys=keys,
                        init_z=z0, num_warmup=0, **out)

    # cholupdate known answers
    rng = np.random.default_rng(11)
    kat = {}
    for d in (1, 3, 8, 26, 64):
        A = rng.normal(size=(d, d))
        L = np.linalg.cholesky(A @ A.T + d * np.eye(d))
        x = rng.normal(size=d)
        for k, gm in enumerate((0.5, 0.01)):
            kat[f"d{d}_{k}_L"] = L
            kat[f"d{d}_{k}_x"] = x
            kat[f"d{d}_{k}_gamma"] = np.float64(gm)
            kat[f"d{d}_{k}_out"] = lit.cholesky_update(np.sqrt(1 - gm) * L, x, gm)
    np.savez_compressed(os.path.join(HERE, "cholupdate.npz"), **kat)


if __name__ == "__main__":
    main()
