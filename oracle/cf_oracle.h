/*
 * cf_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference algorithm
 * (platforms/reference/src/ReferenceCoulKernels.cpp) used as the parity checker.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (libchargeflux_hip.so) never links or calls this code.
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors, and it
 * cannot be built here (it needs OpenMM headers/libraries, which this image lacks).
 * This restatement is pinned only by physics known-answer tests (tests/test_oracle.py:
 * two-charge Coulomb, NaCl Madelung constant, finite-difference forces, charge
 * conservation) — see DESIGN.md §3.
 */
#ifndef CF_ORACLE_H_
#define CF_ORACLE_H_

#include "../include/chargeflux.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfo_state cfo_state;

/* ReferenceCalcCoulForceKernel::initialize (ReferenceCoulKernels.cpp:230-422).
 * Returns NULL on validation failure (message in err). */
cfo_state* cfo_create(const cf_params* p, char* err, int errlen);
void cfo_destroy(cfo_state* s);
int cfo_ewald(const cfo_state* s, double* alpha, int32_t kmax[3]);

/* ReferenceCalcCoulForceKernel::execute (ReferenceCoulKernels.cpp:424-636).
 * forces [N*3] is ADDED to.  terms/q_out/dedq_out may be NULL.
 * Returns the energy exactly as the reference returns it. */
double cfo_execute(cfo_state* s, const double* pos, const double* box9, int include_forces,
                   int include_energy, double* forces, double terms[4], double* q_out,
                   double* dedq_out);

/* execute with the reciprocal loop cut after k_count k-vectors (k_count = 0: none) —
 * used to check the non-reciprocal terms at sizes where the full k-sum is too slow. */
double cfo_execute_klimit(cfo_state* s, const double* pos, const double* box9, int include_forces,
                          int include_energy, double* forces, double terms[4], int64_t k_count);

/* CPU-baseline sampling: time the real-space + flux + chain part of one evaluation
 * fully and the reciprocal half-space loop over only its first k_count k-vectors
 * (same per-k work as the reference: 2 passes x cos+sin per atom).  Returns
 * seconds for each part; *k_total receives the full K_half. */
int cfo_time_sample(cfo_state* s, const double* pos, const double* box9, int64_t k_count,
                    double* t_nonrecip, double* t_recip_sample, int64_t* k_total);

#ifdef __cplusplus
}
#endif
#endif
