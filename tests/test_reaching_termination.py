"""Why the reference's stored reaching-task optima cannot be reproduced by a converged solve:
Ipopt's own termination tests fail at them, by seven orders of magnitude, whatever the multipliers.

The stored solutions (examples/dynamics/reaching_task/result_file/pulse_duration_minimize_muscle_{fatigue,force}.pkl,
extracted as numbers by tests/golden/extract_reaching_solution.py) come from
reaching_task_pulse_duration_optimization.py:117, ``ocp.solve(Solver.IPOPT(_max_iter=10000))``, with the per-pulse
widths as parameters in seconds (VariableScaling 1, cocofest/optimization/fes_ocp_dynamics.py:373).  Ipopt ends a solve
with Solve_Succeeded only when its scaled error is <= tol (bioptim: 1e-6) and the unscaled dual infeasibility <=
dual_inf_tol (1); with Solved_To_Acceptable_Level only when the scaled error is <= acceptable_tol (1e-6) for 15
iterations (IpOptErrorConv).  tests/reaching_kkt.py::ipopt_termination_audit computes, in the stored revision's NLP, the
best multipliers there are (least squares with signed bound multipliers, and a linear program for the smallest max-norm
dual infeasibility any multipliers give) and Ipopt's scaled error with them.  Neither success exit can have ended the
stored solves; the remaining Ipopt exit consistent with their 17,973 s / 11,712 s run times is the script's
_max_iter = 10000 (Maximum_Iterations_Exceeded: the last iterate is returned and pickled).  A converged solve therefore
lands elsewhere ("Optimiser parity")."""

import pytest

from tests import reaching_kkt as K


@pytest.mark.parametrize("objective,dmin", [("fatigue", 40.0), ("force", 5e5)])
def test_stored_optima_fail_ipopts_termination_tests(objective, dmin):
    a = K.ipopt_termination_audit(objective)
    print(objective, {k: a[k] for k in ("dual_inf_unscaled_ls", "dual_inf_unscaled_min_lp", "scaled_error_ls",
                                        "scaled_error_lp", "s_d_ls", "s_d_lp", "at_bounds", "active_kept")})
    assert a["lp_status"] == 0
    # the smallest unscaled dual infeasibility any multipliers give (LP) is far above dual_inf_tol = 1 ...
    assert a["dual_inf_unscaled_min_lp"] > dmin > a["dual_inf_tol"]
    assert a["dual_inf_unscaled_ls"] >= a["dual_inf_unscaled_min_lp"] * (1 - 1e-9)
    # ... and Ipopt's scaled error with those multipliers exceeds tol = acceptable_tol = 1e-6 by more than 10^7 (47.5 for
    # the fatigue optimum, 5.4e3 for the force one): neither Solve_Succeeded nor Solved_To_Acceptable_Level
    assert min(a["scaled_error_ls"], a["scaled_error_lp"]) > 1e7 * a["acceptable_tol"]
