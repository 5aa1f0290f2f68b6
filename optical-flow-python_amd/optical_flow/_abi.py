"""ctypes mirror of include/optflow.h (POD structs and enums only).

Kept free of any library loading so that both the product binding
(optical_flow._native) and the test oracle wrapper (oracle/oracle.py) can
share the exact struct layout.
"""
import ctypes as C

OF_ABI_VERSION = 3

OF_OK, OF_EINVAL, OF_EHIP, OF_ENOMEM, OF_ENOTSUP, OF_ERCCL = 0, -1, -2, -3, -4, -5

METHOD = {"hs": 0, "ba": 1, "classic_nl": 2, "alt_ba": 3}
INTERP = {"cubic": 0, "bi-cubic": 1, "bi-linear": 2}
SOLVER = {"backslash": 0, "pcg": 1, "sor": 2}
PENALTY = {
    "quadratic": 0, "lorentzian": 1, "charbonnier": 2, "generalized_charbonnier": 3,
    "geman_mcclure": 4, "huber": 5, "tukey": 6, "gaussian": 7, "tdist": 8, "tdist_unnorm": 9,
    "const": 100,
}
MAX_LEVELS = 32
OF_OPT_SOR_PIPELINE = 1  # of_set_option
OF_OPT_SOR_FALLBACKS = 2  # of_get_option (read-only counter)
OF_OPT_FUSED_WARP = 3  # of_set_option: warp + assembly in one kernel (default 1)
OF_OPT_DEVICE_BYTES = 4  # of_get_option (read-only): grow-only device bytes of the context and its lanes
OF_OPT_RCCL_NRANKS = 5  # of_get_option (read-only): ranks of the RCCL communicator (ncclCommCount; 0 = none)


class OfPenalty(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad_", C.c_int32), ("p0", C.c_double), ("p1", C.c_double)]


_INT_FIELDS = [
    "method", "solver", "interp", "texture", "fc", "auto_level", "pyramid_levels", "gnc_iters",
    "gnc_pyramid_levels", "max_iters", "max_warping_iters", "max_linear", "pcg_maxiter",
    "sor_max_iters", "limit_update", "median_filter_size", "mf_iter", "use_wmf", "area_hsz",
    "itersLO", "exact_maxiter", "display", "guide_mode", "pad_",
]
_DBL_FIELDS = [
    "lambda_", "lambda_q", "alpha", "pyramid_spacing", "gnc_pyramid_spacing", "pcg_rtol",
    "exact_rtol", "sor_omega", "sor_tol", "blend", "alp", "sigma_i", "sigmaD2", "sigmaS2",
    "lambda2", "lambda3",
]


MAX_FILTERS = 8
MAX_FDIM = 5


class OfFilterSet(C.Structure):
    """of_filter_set: a general spatial_filters list (general = 0: the
    default [[1, -1]], [[1], [-1]] pair)"""
    _fields_ = [("general", C.c_int32), ("n", C.c_int32),
                ("fh", C.c_int32 * MAX_FILTERS), ("fw", C.c_int32 * MAX_FILTERS),
                ("taps", (C.c_double * (MAX_FDIM * MAX_FDIM)) * MAX_FILTERS),
                ("rho_u", OfPenalty * MAX_FILTERS), ("rho_v", OfPenalty * MAX_FILTERS),
                ("qua_u", OfPenalty * MAX_FILTERS), ("qua_v", OfPenalty * MAX_FILTERS)]


class OfParams(C.Structure):
    _fields_ = ([(n, C.c_int32) for n in _INT_FIELDS]
                + [(n, C.c_double) for n in _DBL_FIELDS]
                + [("deriv_filter", C.c_double * 5),
                   ("rho_data", OfPenalty), ("rho_spatial_u", OfPenalty * 2), ("rho_spatial_v", OfPenalty * 2),
                   ("qua_data", OfPenalty), ("qua_spatial_u", OfPenalty * 2), ("qua_spatial_v", OfPenalty * 2),
                   ("rho_couple", OfPenalty), ("filters", OfFilterSet)])


class OfStats(C.Structure):
    _fields_ = [
        ("n_levels", C.c_int32),
        ("level_h", C.c_int32 * MAX_LEVELS),
        ("level_w", C.c_int32 * MAX_LEVELS),
        ("level_stage", C.c_int32 * MAX_LEVELS),
        ("level_ms", C.c_double * MAX_LEVELS),
        ("solves", C.c_int32),
        ("solver_iters_total", C.c_int32),
        ("solver_iters_max", C.c_int32),
        ("solves_not_converged", C.c_int32),
        ("total_ms", C.c_double),
        ("preprocess_ms", C.c_double),
    ]

    def as_dict(self):
        n = self.n_levels
        return {
            "levels": [{"h": self.level_h[i], "w": self.level_w[i], "stage": self.level_stage[i],
                        "ms": self.level_ms[i]} for i in range(n)],
            "solves": self.solves, "solver_iters_total": self.solver_iters_total,
            "solver_iters_max": self.solver_iters_max,
            "solves_not_converged": self.solves_not_converged,
            "total_ms": self.total_ms, "preprocess_ms": self.preprocess_ms,
        }


# of_set_progress (include/optflow.h): events and flags
OF_EV_STAGE, OF_EV_LEVEL, OF_EV_ITER, OF_EV_STAGE_END = 0, 1, 2, 3
OF_PROGRESS_ITER, OF_PROGRESS_FLOW = 1, 2


class OfProgress(C.Structure):
    _fields_ = [("event", C.c_int32), ("stage", C.c_int32), ("level", C.c_int32), ("h", C.c_int32),
                ("w", C.c_int32), ("iter", C.c_int32), ("lin", C.c_int32), ("pad_", C.c_int32),
                ("norm", C.c_double), ("elapsed_s", C.c_double), ("uv", C.POINTER(C.c_float))]


OfProgressFn = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(OfProgress))


class OfCgGeometry(C.Structure):
    _fields_ = [("grid_x", C.c_int32), ("grid_y", C.c_int32), ("rows", C.c_int32), ("bands", C.c_int32),
                ("blocks", C.c_int32), ("strip_cols", C.c_int32)]


class OfSolveRecord(C.Structure):
    _fields_ = [("h", C.c_int32), ("w", C.c_int32), ("solver", C.c_int32), ("iters", C.c_int32),
                ("done", C.c_int32), ("pad_", C.c_int32), ("true_rel", C.c_double), ("est_rel", C.c_double),
                ("true_rel_out", C.c_double)]

    def as_dict(self):
        return {"h": self.h, "w": self.w, "solver": self.solver, "iters": self.iters, "done": self.done,
                "true_rel": self.true_rel, "est_rel": self.est_rel, "true_rel_out": self.true_rel_out}


def penalty(kind, p0=1.0, p1=0.0):
    return OfPenalty(PENALTY[kind], 0, float(p0), float(p1))


def penalty_from_robust(rf):
    """OfPenalty from an optical_flow.robust.RobustFunction (robust_function.py:47-83)."""
    p = list(rf.param) + [0.0]
    return OfPenalty(PENALTY[rf.method], 0, float(p[0]), float(p[1]))
