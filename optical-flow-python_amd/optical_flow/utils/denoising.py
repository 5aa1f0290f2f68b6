"""Li-Osher iterated median (reference: optical_flow/utils/denoising.py:6-30)."""
import numpy as np

from optical_flow.utils.weighted_median import median_filter2


def denoise_LO(un, mfsz, lambda_param, n_iters=1):
    if mfsz is None:
        return np.array(un, dtype=float, copy=True)
    s = (int(mfsz[0]), int(mfsz[1])) if isinstance(mfsz, (list, tuple, np.ndarray)) else (int(mfsz),) * 2
    if s[0] != s[1]:
        raise NotImplementedError("square median sizes only")
    un = np.asarray(un, dtype=float)
    u = un.copy()
    for _ in range(n_iters):
        u = median_filter2(u + lambda_param * (un - u), s[0])
    return u
