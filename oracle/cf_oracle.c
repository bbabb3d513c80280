/*
 * cf_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline "port").
 *
 * Plain-C restatement of the reference's fp64 serial implementation:
 *   platforms/reference/src/ReferenceCoulKernels.cpp (RCK below) and the parameter
 *   container openmmapi/src/CoulForce.cpp.  Each function cites the lines it follows.
 * It is written from the semantics, not copied; loop order of the reciprocal sum and
 * every quirk listed in SURVEY.md Appendix A.3 ("Reproduce") are kept so it can serve
 * as the serial CPU baseline.  Periodic boxes in OpenMM's reduced form a = (ax,0,0),
 * b = (bx,by,0), c = (cx,cy,cz): the minimum image uses the box vectors
 * (getDeltaRPeriodic), the reciprocal part reads only the box diagonals (RCK:513-517).
 *
 * PARITY UNPINNED: see cf_oracle.h.
 */
#include "cf_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

struct cfo_state {
    int n;
    double* charges;   /* q0                                       RCK:237           */
    double* lj;        /* [2N] (sigma/2, 2*sqrt(eps))              RCK:238-239       */
    double* realq;     /* realcharges                              RCK:37-40         */
    int nb, na, nw;
    int* bidx; double* bpar;
    int* aidx; double* apar;
    int* widx; double* wpar;
    int nd;            /* dq/dx entries 4B+9A+9W                   RCK:286-383       */
    int* dq_q; int* dq_x; double* dq_val;
    int* ex_start; int* ex_list; /* per-atom sorted unique exclusion sets RCK:385-391 */
    int pbc;
    double cutoff, tol, alpha, one_alpha2;
    double ke;         /* ONE_4PI_EPS0 of the OpenMM evaluated for (RCK:7; cf_params.one_4pi_eps0) */
    int kmax[3];
};

static void set_err(char* err, int len, const char* msg) {
    if (err && len > 0) { strncpy(err, msg, (size_t)len - 1); err[len - 1] = 0; }
}

/* getEwaldParamValue, RCK:32-35 */
static double ewald_param_value(int kmax, double width, double alpha) {
    double t = kmax * M_PI / (width * alpha);
    return 0.05 * sqrt(width * alpha) * kmax * exp(-t * t);
}

static int cmp_int(const void* a, const void* b) {
    int x = *(const int*)a, y = *(const int*)b;
    return (x > y) - (x < y);
}

/* initialize, RCK:230-422 */
cfo_state* cfo_create(const cf_params* p, char* err, int errlen) {
    int n = p->num_particles;
    if (n <= 0) { set_err(err, errlen, "num_particles must be > 0"); return NULL; }
    cfo_state* s = (cfo_state*)calloc(1, sizeof(cfo_state));
    s->n = n;
    s->charges = (double*)malloc(sizeof(double) * n);
    s->lj = (double*)malloc(sizeof(double) * 2 * n);
    s->realq = (double*)malloc(sizeof(double) * n);
    for (int i = 0; i < n; i++) {
        s->charges[i] = p->charges[i];
        s->lj[2 * i] = 0.5 * p->sigmas[i];                /* RCK:238 */
        s->lj[2 * i + 1] = 2.0 * sqrt(p->epsilons[i]);    /* RCK:239 */
    }
    s->nb = p->num_flux_bonds; s->na = p->num_flux_angles; s->nw = p->num_flux_waters;
    s->bidx = (int*)malloc(sizeof(int) * 2 * (s->nb + 1));
    s->bpar = (double*)malloc(sizeof(double) * 2 * (s->nb + 1));
    s->aidx = (int*)malloc(sizeof(int) * 3 * (s->na + 1));
    s->apar = (double*)malloc(sizeof(double) * 2 * (s->na + 1));
    s->widx = (int*)malloc(sizeof(int) * 3 * (s->nw + 1));
    s->wpar = (double*)malloc(sizeof(double) * 5 * (s->nw + 1));
    if (s->nb) { memcpy(s->bidx, p->flux_bond_idx, sizeof(int) * 2 * s->nb); memcpy(s->bpar, p->flux_bond_params, sizeof(double) * 2 * s->nb); }
    if (s->na) { memcpy(s->aidx, p->flux_angle_idx, sizeof(int) * 3 * s->na); memcpy(s->apar, p->flux_angle_params, sizeof(double) * 2 * s->na); }
    if (s->nw) { memcpy(s->widx, p->flux_water_idx, sizeof(int) * 3 * s->nw); memcpy(s->wpar, p->flux_water_params, sizeof(double) * 5 * s->nw); }
    for (int i = 0; i < 2 * s->nb; i++) if (s->bidx[i] < 0 || s->bidx[i] >= n) { set_err(err, errlen, "flux bond index out of range"); cfo_destroy(s); return NULL; }
    for (int i = 0; i < 3 * s->na; i++) if (s->aidx[i] < 0 || s->aidx[i] >= n) { set_err(err, errlen, "flux angle index out of range"); cfo_destroy(s); return NULL; }
    for (int i = 0; i < 3 * s->nw; i++) if (s->widx[i] < 0 || s->widx[i] >= n) { set_err(err, errlen, "flux water index out of range"); cfo_destroy(s); return NULL; }

    /* dq/dx topology: per term, (q-atom major, x-atom minor)  RCK:286-383 */
    s->nd = 4 * s->nb + 9 * s->na + 9 * s->nw;
    s->dq_q = (int*)malloc(sizeof(int) * (s->nd + 1));
    s->dq_x = (int*)malloc(sizeof(int) * (s->nd + 1));
    s->dq_val = (double*)calloc((size_t)3 * (s->nd + 1), sizeof(double));
    int e = 0;
    for (int t = 0; t < s->nb; t++) {
        int a[2] = {s->bidx[2 * t], s->bidx[2 * t + 1]};
        for (int u = 0; u < 2; u++) for (int v = 0; v < 2; v++) { s->dq_q[e] = a[u]; s->dq_x[e] = a[v]; e++; }
    }
    for (int t = 0; t < s->na; t++) {
        int a[3] = {s->aidx[3 * t], s->aidx[3 * t + 1], s->aidx[3 * t + 2]};
        for (int u = 0; u < 3; u++) for (int v = 0; v < 3; v++) { s->dq_q[e] = a[u]; s->dq_x[e] = a[v]; e++; }
    }
    for (int t = 0; t < s->nw; t++) {
        int a[3] = {s->widx[3 * t], s->widx[3 * t + 1], s->widx[3 * t + 2]};
        for (int u = 0; u < 3; u++) for (int v = 0; v < 3; v++) { s->dq_q[e] = a[u]; s->dq_x[e] = a[v]; e++; }
    }

    /* exclusion sets (std::set semantics: unique, ordered)  RCK:385-391 */
    int ne = p->num_exceptions;
    int* cnt = (int*)calloc((size_t)n + 1, sizeof(int));
    for (int k = 0; k < ne; k++) {
        int p1 = p->exceptions[2 * k], p2 = p->exceptions[2 * k + 1];
        if (p1 < 0 || p1 >= n || p2 < 0 || p2 >= n) { free(cnt); set_err(err, errlen, "exception index out of range"); cfo_destroy(s); return NULL; }
        cnt[p1]++; cnt[p2]++;
    }
    s->ex_start = (int*)malloc(sizeof(int) * (n + 1));
    s->ex_start[0] = 0;
    for (int i = 0; i < n; i++) s->ex_start[i + 1] = s->ex_start[i] + cnt[i];
    int* tmp = (int*)malloc(sizeof(int) * (s->ex_start[n] + 1));
    int* fill = (int*)calloc((size_t)n + 1, sizeof(int));
    for (int k = 0; k < ne; k++) {
        int p1 = p->exceptions[2 * k], p2 = p->exceptions[2 * k + 1];
        tmp[s->ex_start[p1] + fill[p1]++] = p2;
        tmp[s->ex_start[p2] + fill[p2]++] = p1;
    }
    /* sort + unique per atom, compact */
    s->ex_list = (int*)malloc(sizeof(int) * (s->ex_start[n] + 1));
    int w = 0;
    int* newstart = (int*)malloc(sizeof(int) * (n + 1));
    for (int i = 0; i < n; i++) {
        int b = s->ex_start[i], c = s->ex_start[i + 1];
        qsort(tmp + b, (size_t)(c - b), sizeof(int), cmp_int);
        newstart[i] = w;
        for (int k = b; k < c; k++) if (k == b || tmp[k] != tmp[k - 1]) s->ex_list[w++] = tmp[k];
    }
    newstart[n] = w;
    free(s->ex_start); s->ex_start = newstart;
    free(tmp); free(fill); free(cnt);

    if (!(p->one_4pi_eps0 >= 0) || !isfinite(p->one_4pi_eps0)) { set_err(err, errlen, "one_4pi_eps0 must be finite and >= 0"); cfo_destroy(s); return NULL; }
    s->ke = p->one_4pi_eps0 == 0 ? CF_ONE_4PI_EPS0 : p->one_4pi_eps0;
    s->pbc = p->use_pbc ? 1 : 0;
    if (s->pbc) {
        const double* b = p->default_box;
        s->cutoff = p->cutoff;
        s->tol = p->ewald_tol;
        if (!(s->cutoff > 0) || !(s->tol > 0 && s->tol < 0.5)) { set_err(err, errlen, "invalid cutoff or ewald tolerance"); cfo_destroy(s); return NULL; }
        if (b[1] != 0 || b[2] != 0 || b[5] != 0 || !(b[0] > 0 && b[4] > 0 && b[8] > 0) ||
            fabs(b[3]) > 0.5 * b[0] || fabs(b[6]) > 0.5 * b[0] || fabs(b[7]) > 0.5 * b[4]) {
            set_err(err, errlen, "periodic box must be in OpenMM's reduced form"); cfo_destroy(s); return NULL;
        }
        s->alpha = (1.0 / s->cutoff) * sqrt(-log(2.0 * s->tol));  /* RCK:401 */
        s->one_alpha2 = 1.0 / s->alpha / s->alpha;                /* RCK:402 */
        double L[3] = {b[0], b[4], b[8]};
        for (int d = 0; d < 3; d++) {                              /* RCK:403-420 */
            int k = 1;
            while (ewald_param_value(k, L[d], s->alpha) > s->tol) k++;
            if (k % 2 == 0) k++;
            s->kmax[d] = k;
        }
    }
    return s;
}

void cfo_destroy(cfo_state* s) {
    if (!s) return;
    free(s->charges); free(s->lj); free(s->realq);
    free(s->bidx); free(s->bpar); free(s->aidx); free(s->apar); free(s->widx); free(s->wpar);
    free(s->dq_q); free(s->dq_x); free(s->dq_val); free(s->ex_start); free(s->ex_list);
    free(s);
}

int cfo_ewald(const cfo_state* s, double* alpha, int32_t kmax[3]) {
    if (alpha) *alpha = s->alpha;
    if (kmax) { kmax[0] = s->kmax[0]; kmax[1] = s->kmax[1]; kmax[2] = s->kmax[2]; }
    return 0;
}

/* ReferenceForce::getDeltaR / getDeltaRPeriodic (OpenMM): d = J - I, minimum image by the
 * box vectors c, b, a in that order.  L = {ax, by, cz, bx, cx, cy} (off-diagonals 0 for an
 * orthorhombic box: the same bits as the per-axis form). */
static inline void delta_r(const double* pi, const double* pj, const double* L, int pbc, double d[3]) {
    for (int k = 0; k < 3; k++) d[k] = pj[k] - pi[k];
    if (pbc) {
        double sc = floor(d[2] / L[2] + 0.5);
        d[0] -= sc * L[4]; d[1] -= sc * L[5]; d[2] -= sc * L[2];
        double sb = floor(d[1] / L[1] + 0.5);
        d[0] -= sb * L[3]; d[1] -= sb * L[1];
        d[0] -= L[0] * floor(d[0] / L[0] + 0.5);
    }
}

static int is_excluded(const cfo_state* s, int i, int j) {
    for (int k = s->ex_start[i]; k < s->ex_start[i + 1]; k++) if (s->ex_list[k] == j) return 1;
    return 0;
}

/* updateRealCharge, RCK:37-228 */
static void update_real_charge(cfo_state* s, const double* pos, const double* L) {
    int pbc = s->pbc;
    for (int i = 0; i < s->n; i++) s->realq[i] = s->charges[i];
    for (int t = 0; t < s->nb; t++) {                         /* bonds RCK:42-80 */
        int p1 = s->bidx[2 * t], p2 = s->bidx[2 * t + 1];
        double k = s->bpar[2 * t], b = s->bpar[2 * t + 1];
        double d[3]; delta_r(pos + 3 * p1, pos + 3 * p2, L, pbc, d);
        double r = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        double dq = k * (r - b);
        s->realq[p1] += dq; s->realq[p2] -= dq;
        double c = k / r;
        double* v = s->dq_val + 3 * (4 * t);
        for (int j = 0; j < 3; j++) {
            double val = c * d[j];
            v[j] = -val; v[3 + j] = val; v[6 + j] = val; v[9 + j] = -val;
        }
    }
    for (int t = 0; t < s->na; t++) {                         /* angles RCK:81-162 */
        int p1 = s->aidx[3 * t], p2 = s->aidx[3 * t + 1], p3 = s->aidx[3 * t + 2];
        double k = s->apar[2 * t], th0 = s->apar[2 * t + 1];
        double d21[3], d23[3], d13[3];
        delta_r(pos + 3 * p2, pos + 3 * p1, L, pbc, d21);
        delta_r(pos + 3 * p2, pos + 3 * p3, L, pbc, d23);
        delta_r(pos + 3 * p1, pos + 3 * p3, L, pbc, d13);
        double r21_2 = d21[0] * d21[0] + d21[1] * d21[1] + d21[2] * d21[2];
        double r23_2 = d23[0] * d23[0] + d23[1] * d23[1] + d23[2] * d23[2];
        double r13_2 = d13[0] * d13[0] + d13[1] * d13[1] + d13[2] * d13[2];
        double r21 = sqrt(r21_2), r23 = sqrt(r23_2);
        double cost = (r23_2 + r21_2 - r13_2) / 2 / r21 / r23;
        double dq = k * (acos(cost) - th0);
        s->realq[p1] += dq; s->realq[p3] += dq; s->realq[p2] -= 2 * dq;
        double inv_s = 1 / sqrt(1 - cost * cost);
        double c1 = k * (1.0 / r21 / r23) * inv_s;
        double c21 = k * cost * inv_s / r21_2;
        double c23 = k * cost * inv_s / r23_2;
        double* v = s->dq_val + 3 * (4 * s->nb + 9 * t);
        for (int j = 0; j < 3; j++) {
            double v1 = -c1 * d23[j] + c21 * d21[j];
            double v3 = -c1 * d21[j] + c23 * d23[j];
            double v2 = -v1 - v3;
            v[0 + j] = v1; v[3 + j] = v2; v[6 + j] = v3;
            v[9 + j] = -2 * v1; v[12 + j] = -2 * v2; v[15 + j] = -2 * v3;
            v[18 + j] = v1; v[21 + j] = v2; v[24 + j] = v3;
        }
    }
    for (int t = 0; t < s->nw; t++) {                         /* waters RCK:163-227 */
        int p1 = s->widx[3 * t], p2 = s->widx[3 * t + 1], p3 = s->widx[3 * t + 2];
        const double* w = s->wpar + 5 * t;
        double k1 = w[0], k2 = w[1], kub = w[2], b0 = w[3], ub0 = w[4];
        double d12[3], d13[3], d23[3];
        delta_r(pos + 3 * p1, pos + 3 * p2, L, pbc, d12);
        delta_r(pos + 3 * p1, pos + 3 * p3, L, pbc, d13);
        delta_r(pos + 3 * p2, pos + 3 * p3, L, pbc, d23);
        double r12 = sqrt(d12[0] * d12[0] + d12[1] * d12[1] + d12[2] * d12[2]);
        double r13 = sqrt(d13[0] * d13[0] + d13[1] * d13[1] + d13[2] * d13[2]);
        double r23 = sqrt(d23[0] * d23[0] + d23[1] * d23[1] + d23[2] * d23[2]);
        double dq2 = k1 * (r12 - b0) + k2 * (r13 - b0) + kub * (r23 - ub0);
        double dq3 = k1 * (r13 - b0) + k2 * (r12 - b0) + kub * (r23 - ub0);
        double dq1 = -dq2 - dq3;
        s->realq[p1] += dq1; s->realq[p2] += dq2; s->realq[p3] += dq3;
        double* v = s->dq_val + 3 * (4 * s->nb + 9 * s->na + 9 * t);
        for (int j = 0; j < 3; j++) {
            double n12 = d12[j] / r12, n13 = d13[j] / r13, n23 = d23[j] / r23;
            double a12k1 = k1 * n12, a12k2 = k2 * n12, a13k1 = k1 * n13, a13k2 = k2 * n13, ub = kub * n23;
            v[0 + j] = a12k1 + a12k2 + a13k1 + a13k2;
            v[3 + j] = -a12k1 - a12k2 + 2 * ub;
            v[6 + j] = -a13k2 - a13k1 - 2 * ub;
            v[9 + j] = -a12k1 - a13k2;
            v[12 + j] = a12k1 - ub;
            v[15 + j] = a13k2 + ub;
            v[18 + j] = -a12k2 - a13k1;
            v[21 + j] = a12k2 - ub;
            v[24 + j] = a13k1 + ub;
        }
    }
}

/* LJ pair of the reference: eps'_i eps'_j s^6 (s^6 - 1), s = (sig'_i + sig'_j)/r  RCK:572-577 */
static inline void lj_terms(const cfo_state* s, int i, int j, double inv_r, double* sig6, double* epssig6) {
    double sig = s->lj[2 * i] + s->lj[2 * j];
    double s2 = inv_r * sig; s2 *= s2;
    *sig6 = s2 * s2 * s2;
    *epssig6 = *sig6 * s->lj[2 * i + 1] * s->lj[2 * j + 1];
}

/* O(N) cell-list stand-in for OpenMM computeNeighborListVoxelHash (RCK:559): every
 * non-excluded pair i<j with minimum-image r^2 <= rc^2 is visited once. */
typedef void (*pair_fn)(cfo_state*, int, int, const double*, const double*, void*);

static void for_each_pair(cfo_state* s, const double* pos, const double* L, pair_fn fn, void* ctx) {
    int n = s->n;
    double rc = s->cutoff, rc2 = rc * rc;
    int nc[3];
    for (int d = 0; d < 3; d++) { nc[d] = (int)floor(L[d] / rc); if (nc[d] < 1) nc[d] = 1; }
    const int triclinic = L[3] != 0 || L[4] != 0 || L[5] != 0;   /* all pairs (small test systems) */
    if (triclinic || nc[0] < 3 || nc[1] < 3 || nc[2] < 3) {
        for (int i = 0; i < n; i++)
            for (int j = i + 1; j < n; j++) {
                double d[3]; delta_r(pos + 3 * j, pos + 3 * i, L, 1, d);
                double r2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
                if (r2 <= rc2 && !is_excluded(s, i, j)) fn(s, i, j, pos, L, ctx);
            }
        return;
    }
    int ncell = nc[0] * nc[1] * nc[2];
    int* head = (int*)malloc(sizeof(int) * ncell);
    int* next = (int*)malloc(sizeof(int) * n);
    int* cell = (int*)malloc(sizeof(int) * n);
    for (int c = 0; c < ncell; c++) head[c] = -1;
    for (int i = n - 1; i >= 0; i--) {
        int ci[3];
        for (int d = 0; d < 3; d++) {
            double x = pos[3 * i + d] - floor(pos[3 * i + d] / L[d]) * L[d];
            int c = (int)(x / L[d] * nc[d]);
            if (c >= nc[d]) c = nc[d] - 1;
            if (c < 0) c = 0;
            ci[d] = c;
        }
        int c = (ci[0] * nc[1] + ci[1]) * nc[2] + ci[2];
        cell[i] = c; next[i] = head[c]; head[c] = i;
    }
    for (int i = 0; i < n; i++) {
        int c = cell[i];
        int cx = c / (nc[1] * nc[2]), cy = (c / nc[2]) % nc[1], cz = c % nc[2];
        for (int ox = -1; ox <= 1; ox++)
            for (int oy = -1; oy <= 1; oy++)
                for (int oz = -1; oz <= 1; oz++) {
                    int x = (cx + ox + nc[0]) % nc[0], y = (cy + oy + nc[1]) % nc[1], z = (cz + oz + nc[2]) % nc[2];
                    for (int j = head[(x * nc[1] + y) * nc[2] + z]; j >= 0; j = next[j]) {
                        if (j <= i) continue;
                        double d[3]; delta_r(pos + 3 * j, pos + 3 * i, L, 1, d);
                        double r2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
                        if (r2 <= rc2 && !is_excluded(s, i, j)) fn(s, i, j, pos, L, ctx);
                    }
                }
    }
    free(head); free(next); free(cell);
}

typedef struct {
    double* forces; double* dedq; double energy; int include_forces;
} real_ctx;

/* real-space pair, RCK:562-593 */
static void real_pair(cfo_state* s, int ii, int jj, const double* pos, const double* L, void* vctx) {
    real_ctx* c = (real_ctx*)vctx;
    double d[3]; delta_r(pos + 3 * jj, pos + 3 * ii, L, 1, d);   /* pos[ii]-pos[jj] */
    double r = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    double inv_r = 1.0 / r, ar = s->alpha * r;
    double sig6, es6; lj_terms(s, ii, jj, inv_r, &sig6, &es6);
    double qi = s->realq[ii], qj = s->realq[jj];
    double erfc_ar = erfc(ar);
    if (c->include_forces) {
        double dEdR = s->ke * qi * qj * inv_r * inv_r * inv_r;
        dEdR *= erfc_ar + ar * exp(-ar * ar) * 2.0 / sqrt(M_PI);
        dEdR += es6 * (12 * sig6 - 6) * inv_r * inv_r;
        for (int k = 0; k < 3; k++) {
            double f = dEdR * d[k];
            c->forces[3 * ii + k] += f; c->forces[3 * jj + k] -= f;
        }
        c->dedq[ii] += s->ke * qj * inv_r * erfc_ar;
        c->dedq[jj] += s->ke * qi * inv_r * erfc_ar;
    }
    c->energy += s->ke * qi * qj * inv_r * erfc_ar + es6 * (sig6 - 1);
}

/* reciprocal half-space loop, RCK:513-556.  Visits k-vectors [k_lo, k_hi) of the
 * reference's visiting order (k_hi < 0: all). Returns the number visited. */
static int64_t recip_sum(cfo_state* s, const double* pos, const double* L, int include_forces,
                         int include_energy, double* forces, double* dedq, double* e_recip,
                         int64_t k_hi) {
    int n = s->n;
    double rx = 2 * M_PI / L[0], ry = 2 * M_PI / L[1], rz = 2 * M_PI / L[2];
    double constant = 4.0 / L[0] / L[1] / L[2] * M_PI * s->ke;   /* RCK:517 */
    double energy = 0;
    int64_t visited = 0;
    int minky = 0, minkz = 1;
    for (int nkx = 0; nkx < s->kmax[0]; nkx++) {
        double kx = nkx * rx;
        for (int nky = minky; nky < s->kmax[1]; nky++) {
            double ky = nky * ry;
            for (int nkz = minkz; nkz < s->kmax[2]; nkz++) {
                if (k_hi >= 0 && visited >= k_hi) goto done;
                visited++;
                double kz = nkz * rz;
                double k2 = kx * kx + ky * ky + kz * kz;
                double eak = exp(-k2 * 0.25 * s->one_alpha2) / k2;
                double ss = 0, cs = 0;
                if (include_forces || include_energy) {
                    for (int i = 0; i < n; i++) {
                        double gr = kx * pos[3 * i] + ky * pos[3 * i + 1] + kz * pos[3 * i + 2];
                        cs += s->realq[i] * cos(gr);
                        ss += s->realq[i] * sin(gr);
                    }
                }
                if (include_forces) {
                    for (int i = 0; i < n; i++) {
                        double gr = kx * pos[3 * i] + ky * pos[3 * i + 1] + kz * pos[3 * i + 2];
                        double q = s->realq[i];
                        double gradr = 2.0 * constant * eak * (ss * q * cos(gr) - cs * q * sin(gr));
                        forces[3 * i] -= gradr * kx;
                        forces[3 * i + 1] -= gradr * ky;
                        forces[3 * i + 2] -= gradr * kz;
                        dedq[i] += 2 * constant * eak * (cs * cos(gr) + ss * sin(gr));
                    }
                }
                if (include_energy) energy += constant * eak * (cs * cs + ss * ss);
            }
            minkz = 1 - s->kmax[2];
        }
        minky = 1 - s->kmax[1];
    }
done:
    *e_recip = energy;
    return visited;
}

static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* execute, RCK:424-636.  kspace_limit<0: full k loop; otherwise stop after that many
 * k-vectors (used only for bounded CPU-baseline timing). */
static double execute_impl(cfo_state* s, const double* pos, const double* box9, int include_forces,
                           int include_energy, double* forces, double terms[4], double* dedq_out,
                           int64_t kspace_limit, double* t_nonrecip, double* t_recip) {
    int n = s->n;
    double L[6] = {1, 1, 1, 0, 0, 0};
    if (s->pbc) { L[0] = box9[0]; L[1] = box9[4]; L[2] = box9[8]; L[3] = box9[3]; L[4] = box9[6]; L[5] = box9[7]; }
    double t0 = now_s();
    update_real_charge(s, pos, L);                                  /* RCK:429 */
    double* dedq = (double*)calloc((size_t)n, sizeof(double));
    double energy = 0;
    if (terms) terms[0] = terms[1] = terms[2] = terms[3] = 0;
    if (!s->pbc) {
        /* all pairs, then subtract the exclusions (RCK:436-491) */
        for (int ii = 0; ii < n; ii++)
            for (int jj = ii + 1; jj < n; jj++) {
                double d[3]; delta_r(pos + 3 * ii, pos + 3 * jj, L, 0, d);   /* pos[jj]-pos[ii] */
                double inv_r = 1.0 / sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                double sig6, es6; lj_terms(s, ii, jj, inv_r, &sig6, &es6);
                double qq = s->ke * s->realq[ii] * s->realq[jj] * inv_r;
                if (include_energy) { energy += qq; energy += es6 * (sig6 - 1); }
                if (include_forces) {
                    double dEdR = (es6 * (12 * sig6 - 6) + qq) * inv_r * inv_r;
                    for (int k = 0; k < 3; k++) { forces[3 * ii + k] -= dEdR * d[k]; forces[3 * jj + k] += dEdR * d[k]; }
                    dedq[ii] += s->ke * s->realq[jj] * inv_r;
                    dedq[jj] += s->ke * s->realq[ii] * inv_r;
                }
            }
        for (int p1 = 0; p1 < n; p1++)
            for (int k = s->ex_start[p1]; k < s->ex_start[p1 + 1]; k++) {
                int p2 = s->ex_list[k];
                if (p1 >= p2) continue;
                double d[3]; delta_r(pos + 3 * p1, pos + 3 * p2, L, 0, d);
                double inv_r = 1.0 / sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                double sig6, es6; lj_terms(s, p1, p2, inv_r, &sig6, &es6);
                double qq = s->ke * s->realq[p1] * s->realq[p2] * inv_r;
                if (include_energy) { energy -= qq; energy -= es6 * (sig6 - 1); }
                if (include_forces) {
                    double dEdR = (es6 * (12 * sig6 - 6) + qq) * inv_r * inv_r;
                    for (int c = 0; c < 3; c++) { forces[3 * p1 + c] += dEdR * d[c]; forces[3 * p2 + c] -= dEdR * d[c]; }
                    dedq[p1] -= s->ke * s->realq[p2] * inv_r;
                    dedq[p2] -= s->ke * s->realq[p1] * inv_r;
                }
            }
        if (terms) terms[2] = energy;
    } else {
        double e_self = 0, e_recip = 0, e_real = 0, e_excl = 0;
        for (int i = 0; i < n; i++) {                                   /* RCK:507-510 */
            e_self -= s->ke * s->realq[i] * s->realq[i] * s->alpha / sqrt(M_PI);
            dedq[i] += -2 * s->ke * s->alpha / sqrt(M_PI) * s->realq[i];
        }
        double t1 = now_s();
        recip_sum(s, pos, L, include_forces, include_energy, forces, dedq, &e_recip, kspace_limit);
        double t2 = now_s();
        if (t_recip) *t_recip = t2 - t1;
        real_ctx rc = {forces, dedq, 0.0, include_forces};
        for_each_pair(s, pos, L, real_pair, &rc);                      /* RCK:559-593 */
        e_real = rc.energy;
        for (int p1 = 0; p1 < n; p1++)                                  /* RCK:596-622 */
            for (int k = s->ex_start[p1]; k < s->ex_start[p1 + 1]; k++) {
                int p2 = s->ex_list[k];
                if (p1 >= p2) continue;
                double d[3]; delta_r(pos + 3 * p2, pos + 3 * p1, L, 1, d);   /* pos[p1]-pos[p2] */
                double r = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                double inv_r = 1.0 / r, ar = s->alpha * r;
                double erf_ar = erf(ar);
                if (include_forces) {
                    double dEdR = s->ke * s->realq[p1] * s->realq[p2] * inv_r * inv_r * inv_r;
                    dEdR *= erf_ar - ar * exp(-ar * ar) * 2.0 / sqrt(M_PI);
                    for (int c = 0; c < 3; c++) { forces[3 * p1 + c] -= dEdR * d[c]; forces[3 * p2 + c] += dEdR * d[c]; }
                    dedq[p1] -= s->ke * s->realq[p2] * inv_r * erf_ar;
                    dedq[p2] -= s->ke * s->realq[p1] * inv_r * erf_ar;
                }
                e_excl -= s->ke * s->realq[p1] * s->realq[p2] * inv_r * erf_ar;
            }
        energy = e_self + e_recip + e_real + e_excl;                    /* RCK:633 */
        if (terms) { terms[0] = e_self; terms[1] = e_recip; terms[2] = e_real; terms[3] = e_excl; }
        if (t_nonrecip) *t_nonrecip = (t1 - t0);
    }
    /* chain rule F_x -= dE/dq * dq/dx  (RCK:493-499, 626-632) */
    double tc = now_s();
    for (int e = 0; e < s->nd; e++) {
        int p1 = s->dq_q[e], p2 = s->dq_x[e];
        for (int j = 0; j < 3; j++) forces[3 * p2 + j] -= dedq[p1] * s->dq_val[3 * e + j];
    }
    if (t_nonrecip && s->pbc) *t_nonrecip += now_s() - tc;
    if (dedq_out) memcpy(dedq_out, dedq, sizeof(double) * n);
    free(dedq);
    return energy;
}

double cfo_execute(cfo_state* s, const double* pos, const double* box9, int include_forces,
                   int include_energy, double* forces, double terms[4], double* q_out,
                   double* dedq_out) {
    double e = execute_impl(s, pos, box9, include_forces, include_energy, forces, terms, dedq_out,
                            -1, NULL, NULL);
    if (q_out) memcpy(q_out, s->realq, sizeof(double) * s->n);
    return e;
}

double cfo_execute_klimit(cfo_state* s, const double* pos, const double* box9, int include_forces,
                          int include_energy, double* forces, double terms[4], int64_t k_count) {
    return execute_impl(s, pos, box9, include_forces, include_energy, forces, terms, NULL, k_count, NULL, NULL);
}

int cfo_time_sample(cfo_state* s, const double* pos, const double* box9, int64_t k_count,
                    double* t_nonrecip, double* t_recip_sample, int64_t* k_total) {
    if (!s->pbc) return -1;
    int kx = s->kmax[0], ky = s->kmax[1], kz = s->kmax[2];
    *k_total = (int64_t)(kz - 1) + (int64_t)(ky - 1) * (2 * kz - 1) + (int64_t)(kx - 1) * (2 * ky - 1) * (2 * kz - 1);
    double* f = (double*)calloc((size_t)3 * s->n, sizeof(double));
    double tn = 0, tr = 0;
    double t_start = now_s();
    execute_impl(s, pos, box9, 1, 1, f, NULL, NULL, k_count, &tn, &tr);
    double t_all = now_s() - t_start;
    *t_nonrecip = t_all - tr;
    *t_recip_sample = tr;
    free(f);
    return 0;
}
