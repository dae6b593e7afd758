// ppls_xprod.h -- launch interface of the cross-product form of the PPLS_simult iteration
// (ppls_xprod.hip; the joint Gram lives with the other MFMA Gram in ppls_variances.hip).
//
// Every data-dependent quantity of one EM iteration is a quadratic form in the
// joint cross-product S = [X Y]'[X Y]: with B = blockdiag(W, C) and M = S B,
//   X'mu_T = X'X W diag(alpha) + X'Y C diag(beta)  = M[X rows] (alpha | beta)      (:732, :691-692)
//   Y'mu_U = Y'X W diag(gamma) + Y'Y C diag(delta) = M[Y rows] (gamma | delta)     (:733, :693-694)
//   Gram([Xw Yc]) = B' M                                                           (:696-712, loglC.cpp:335)
// so once S is formed (one MFMA-bound pass over the data), an iteration reads S, not X and Y.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppls_math.h"

extern "C" {
// Gram of the joint column space [X | Y] (xcols columns of X at stride ldx, then ycols of Y at
// stride ldy; both multiples of the 16-B vector; xreal / yreal of them real, the rest zero padding):
// every live 64 x 64 quadrant of the lower 128 x 128 tiles, per row split, into part
// (ppls_gram_part_doubles), by persistent waves taking items from `queue` (ppls_gram_queue_ints(p,
// nsplit) device ints, filled once by ppls_gram_queue_prepare); ppls_launch_gram_finish sums and
// mirrors them.
hipError_t ppls_launch_gram_joint(const void* X, int ldx, int xcols, int xreal, const void* Y, int ldy, int ycols,
                                  int yreal, int f32, int64_t n, int p, int nsplit, double* part, int* queue,
                                  hipStream_t st);

// Rows of S per wave of the tile kernel (rw_opt 1, 2, 4 or 8 (r <= 8) forces it; 0 = auto).
int ppls_xprod_tile_rows(int P, int r, int rw_opt, int num_cus);

// One iteration's statistics from S (P x P row-major, P = ldx + ldy, symmetric) and theta = (Wp, Cp,
// sc): stats = [X'mu_T (ldx x r) | Y'mu_U (ldy x r) | Gram (2r x 2r)], the layout the sweeps'
// reduction writes.  The tile kernel (rw rows of S per wave) streams S once and writes the X'mu_T,
// Y'mu_U rows and M = S B (P x 2r column-major, scratch); the Gram kernel forms B'M, one workgroup
// per entry (fixed-order sums: deterministic) -- unless with_gram = 0, when the finalize that
// follows forms it (PplsFinalizeArgs::xpM, r <= 8).
// stop: the em_run stop flag (both kernels exit if it is set) or nullptr.
hipError_t ppls_launch_xprod_tile(const double* S, int ldx, int ldy, int r, int rw, const double* Wp,
                                  const double* Cp, const PplsScalars* sc, double* stats, double* M, const int* stop,
                                  int with_gram, hipStream_t st);

}
