"""Accuracy of the stage-chain factorisation on ill-conditioned KKT-shaped systems, for the library given by CFX_LIB
(A/B of two builds): symmetric blocks [[H + Sigma, J^T], [J, -1e-9 I]] with Sigma spanning 1e-8 .. 1e10 (an interior
point near a degenerate optimum), couplings L_k = U_{k-1}^T.  Reports the relative residual and the error against
numpy's dense solve (long double refinement unavailable: the dense solve is the reference).  Usage (GPU):
CFX_LIB=... python scripts/chain_accuracy_ab.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_chain_kkt import _btri, _dense  # noqa: E402

out = []
for seed in range(6):
    rng = np.random.default_rng(seed)
    B, M, sp = 1, 40, 80
    nr = 34
    D = np.zeros((B, M, sp, sp))
    for k in range(M):
        H = rng.normal(size=(sp - nr, sp - nr))
        H = 0.5 * (H + H.T)
        sig = 10.0 ** rng.uniform(-8, 10, sp - nr)
        J = rng.normal(size=(nr, sp - nr))
        D[0, k, : sp - nr, : sp - nr] = H + np.diag(sig)
        D[0, k, sp - nr:, : sp - nr] = J
        D[0, k, : sp - nr, sp - nr:] = J.T
        D[0, k, sp - nr:, sp - nr:] = -1e-9 * np.eye(nr)
    U = 0.5 * rng.normal(size=(B, M, sp, sp))
    U[:, M - 1] = 0.0
    L = np.zeros_like(U)
    L[:, 1:] = np.transpose(U[:, :-1], (0, 1, 3, 2))
    rhs = rng.normal(size=(B, 1, M * sp))
    x, info = _btri(D, L, U, rhs)
    A = _dense(D, L, U, 0)
    ref = np.linalg.solve(A, rhs[0].T).T
    res = np.abs(x[0] @ A.T - rhs[0]).max() / (np.abs(A).max() * np.abs(x[0]).max())
    out.append({"seed": seed, "info": int(info[0]), "rel_residual": float(res),
                "rel_err_vs_dense": float(np.abs(x[0] - ref).max() / np.abs(ref).max())})
print(json.dumps({"lib": os.environ.get("CFX_LIB", "libcfx.so"), "cases": out,
                  "residual_max": max(c["rel_residual"] for c in out), "err_max": max(c["rel_err_vs_dense"] for c in out)}))
