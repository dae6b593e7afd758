"""ppls_amd -- MI355X-native (gfx950) EM inner loop of PPLS_simult (selbouhaddani/PPLS).

The product is the C-ABI library ``libppls_amd.so`` (include/ppls.h, HIP kernels in csrc/);
this package is its Python host binding plus the mirror of the reference's R interface.
"""
from ._lib import PPLS_ORTH_QR, PPLS_ORTH_SVD, Expect, PplsError, Theta  # noqa: F401
from .api import (PPLS, Context, Expect_M, Maximiz_M, PPLS_simult, PPLS_simult_to_o2m, PPLS_to_o2m, PPLSi,  # noqa: F401
                  default_context, fconstraint, initial_guess, logl_W, loglC_fast, meta_EMstep, meta_PPLSi,
                  print_PPLS, random_theta0, scores_PPLS, variances_PPLS_simult)

__all__ = ["Context", "fconstraint", "Expect_M", "Maximiz_M", "PPLS_simult", "PPLS", "PPLSi", "initial_guess", "print_PPLS", "scores_PPLS",
           "PPLS_simult_to_o2m", "PPLS_to_o2m", "meta_EMstep", "meta_PPLSi", "variances_PPLS_simult", "logl_W", "loglC_fast", "Theta",
           "Expect", "PplsError", "random_theta0", "default_context", "PPLS_ORTH_SVD", "PPLS_ORTH_QR"]
