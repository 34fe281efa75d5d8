"""numpy dtypes that mirror the C structs of include/amc_lba.h byte for byte.

Used both by the ctypes binding of the product (`amc_lba.Problem`) and by the oracle
binding under oracle/ (test infrastructure), so both sides read identical buffers.
"""
import ctypes

import numpy as np

KF_DTYPE = np.dtype([
    ("q", "<f8", (4,)), ("t", "<f8", (3,)), ("vel", "<f8", (6,)),
    ("time", "<f8"), ("bf", "<f8"), ("fixed", "<i4"), ("pad", "<i4"),
], align=True)

OBS_DTYPE = np.dtype([
    ("kind", "<i4"), ("kf_a", "<i4"), ("kf_b", "<i4"), ("lm", "<i4"), ("cam", "<i4"), ("pad", "<i4"),
    ("t", "<f8"), ("z", "<f8", (3,)), ("w", "<f8"),
], align=True)

PRIOR_DTYPE = np.dtype([("kf_a", "<i4"), ("kf_b", "<i4")], align=True)

CAM_DTYPE = np.dtype([
    ("q", "<f8", (4,)), ("t", "<f8", (3,)),
    ("fx", "<f8"), ("fy", "<f8"), ("cx", "<f8"), ("cy", "<f8"),
    ("ext_free", "<i4"), ("pad", "<i4"), ("rbc_ini", "<f8", (4,)), ("rbc_info", "<f8", (9,)),
], align=True)

assert KF_DTYPE.itemsize == 128
assert OBS_DTYPE.itemsize == 64
assert PRIOR_DTYPE.itemsize == 8
assert CAM_DTYPE.itemsize == 200

# observation kinds (LBA_MONO_GP ... LBA_STEREO)
MONO_GP, STEREO_GP, MONO, STEREO = 0, 1, 2, 3

# status codes
LBA_OK, LBA_E_EMPTY, LBA_E_SOLVE, LBA_E_DIVERGED, LBA_E_ARG, LBA_E_HIP, LBA_E_LIMIT = 0, -1, -2, -3, -4, -5, -6
LBA_E_TIMEOUT = -7


class LbaConfig(ctypes.Structure):
    _fields_ = [
        ("qc", ctypes.c_double * 36),
        ("huber_mono", ctypes.c_double),
        ("huber_stereo", ctypes.c_double),
        ("huber_prior", ctypes.c_double),
        ("lambda_init", ctypes.c_double),
        ("tau", ctypes.c_double),
        ("max_trials", ctypes.c_int32),
        ("early_stop", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("flags", ctypes.c_int32),
    ]


class LbaStats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int32),
        ("trials", ctypes.c_int32),
        ("result", ctypes.c_int32),
        ("solve_failures", ctypes.c_int32),
        ("chi2_initial", ctypes.c_double),
        ("chi2_final", ctypes.c_double),
        ("lambda_final", ctypes.c_double),
        ("ms_linearize", ctypes.c_double),
        ("ms_schur", ctypes.c_double),
        ("ms_solve", ctypes.c_double),
        ("ms_update_eval", ctypes.c_double),
        ("ms_total", ctypes.c_double),
        ("ms_k_linearize", ctypes.c_double),
        ("n_k_linearize", ctypes.c_int32),
        ("n_k_solve", ctypes.c_int32),
        ("ms_k_solve", ctypes.c_double),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# lba_config.flags (include/amc_lba.h)
FLAG_TIME_SWEEP = 1
FLAG_TIME_PHASES = 2
FLAG_HOST_LOOP = 4         # host-driven LM loop (default: queued trials decided on the device)
FLAG_BAND_SOLVE = 8        # reduced system solved by substitution after the factorisation (large systems)
FLAG_DENSE_SOLVE = 16      # force the L^-1-tile solve
FLAG_TIME_SAMPLED = 32     # with FLAG_TIME_SWEEP (queued loop): events on every 10th trial only
FLAG_SUBTREE_SOLVE = 64    # partitioned: distributed factorisation (window split by lba_partition_assign)
FLAG_F32_RESIDUAL = 128    # per-observation projection / residual / Jacobian rows in fp32, sums in fp64


def make_config(qc_diag=(0.02, 0.02, 0.02, 0.002, 0.002, 0.002), huber_mono=None, huber_stereo=None,
                huber_prior=0.0, lambda_init=1.0, tau=1e-5, max_trials=10, early_stop=1, device=0, flags=0):
    """LocalGPBA defaults: Huber deltas are float sqrt(5.991)/sqrt(7.815) widened to double
    (src/Optimizer.cc:975-978), lambda0 = 1.0 (:848-856), tau 1e-5, 10 trials."""
    cfg = LbaConfig()
    qc = np.zeros((6, 6))
    if np.ndim(qc_diag) == 2:
        qc[:] = qc_diag
    else:
        qc[np.diag_indices(6)] = qc_diag
    for i, v in enumerate(qc.ravel()):
        cfg.qc[i] = float(v)
    cfg.huber_mono = float(np.float32(np.sqrt(5.991))) if huber_mono is None else huber_mono
    cfg.huber_stereo = float(np.float32(np.sqrt(7.815))) if huber_stereo is None else huber_stereo
    cfg.huber_prior = huber_prior
    cfg.lambda_init = lambda_init
    cfg.tau = tau
    cfg.max_trials = max_trials
    cfg.early_stop = early_stop
    cfg.device = device
    cfg.flags = flags
    return cfg


def ptr(a, ctype=ctypes.c_void_p):
    """ctypes pointer to a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctype)
