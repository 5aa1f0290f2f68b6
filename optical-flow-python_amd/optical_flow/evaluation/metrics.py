"""AAE / AEPE (host-side; reference: optical_flow/evaluation/metrics.py:5-53)."""
import numpy as np


def flow_angular_error(tu, tv, u, v, border=0):
    """(mean angular error in degrees, its std, mean end-point error);
    |gt| >= 1e9 marks unknown flow (Middlebury)."""
    tu, tv, u, v = (np.asarray(a, dtype=float) for a in (tu, tv, u, v))
    if border > 0:
        sl = (slice(border, -border), slice(border, -border))
        tu, tv, u, v = tu[sl], tv[sl], u[sl], v[sl]
    ok = (np.abs(tu) < 1e9) & (np.abs(tv) < 1e9)
    if not np.all(ok):
        tu, tv, u, v = tu[ok], tv[ok], u[ok], v[ok]
    cosang = (u * tu + v * tv + 1.0) / (np.sqrt(u * u + v * v + 1.0) * np.sqrt(tu * tu + tv * tv + 1.0))
    ae = np.degrees(np.arccos(np.clip(cosang, -1.0, 1.0)))
    epe = np.sqrt((tu - u) ** 2 + (tv - v) ** 2)
    return np.mean(ae), np.std(ae), np.mean(epe)
