/*
 * fpldpc_oracle.c -- CPU restatement of the reference fixed-point LDPC decode path.
 *
 * TEST INFRASTRUCTURE ONLY (see fpldpc_oracle.h).  Plain C, written from the reference's
 * behaviour (file:line cited per function), deliberately in the reference's own serial shape
 * (banked edge RAM, forward/backward fold, addr_count bank selection) so that it doubles as
 * an honest single-core CPU baseline ("kind": "port" in bench.py).
 */
#include "fpldpc_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ code (ReadH) */
/* ArrayLDPC_Decoder.cpp:642-674: vnum cnum vdeg_max cdeg_max, vdeg[], cdeg[], vlist rows,
 * clist rows, whitespace separated, 0-based. */
int orc_code_load_alist(const char *path, orc_code *c)
{
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    memset(c, 0, sizeof(*c));
    if (fscanf(f, "%d %d %d %d", &c->n, &c->m, &c->dv_max, &c->dc_max) != 4) { fclose(f); return -2; }
    if (c->n <= 0 || c->m <= 0 || c->dv_max <= 0 || c->dc_max <= 0) { fclose(f); return -2; }
    c->vdeg = (int *)calloc(c->n, sizeof(int));
    c->cdeg = (int *)calloc(c->m, sizeof(int));
    c->vlist = (int *)calloc((size_t)c->n * c->dv_max, sizeof(int));
    c->clist = (int *)calloc((size_t)c->m * c->dc_max, sizeof(int));
    int ok = 1;
    for (int i = 0; i < c->n && ok; i++) ok = fscanf(f, "%d", &c->vdeg[i]) == 1 && c->vdeg[i] <= c->dv_max;
    for (int i = 0; i < c->m && ok; i++) ok = fscanf(f, "%d", &c->cdeg[i]) == 1 && c->cdeg[i] <= c->dc_max;
    for (int i = 0; i < c->n && ok; i++)
        for (int j = 0; j < c->vdeg[i] && ok; j++) ok = fscanf(f, "%d", &c->vlist[i * c->dv_max + j]) == 1;
    for (int i = 0; i < c->m && ok; i++)
        for (int j = 0; j < c->cdeg[i] && ok; j++) ok = fscanf(f, "%d", &c->clist[i * c->dc_max + j]) == 1;
    fclose(f);
    if (!ok) { orc_code_free(c); return -3; }
    return 0;
}

void orc_code_free(orc_code *c)
{
    free(c->vdeg); free(c->cdeg); free(c->vlist); free(c->clist);
    memset(c, 0, sizeof(*c));
}

/* ------------------------------------------------------------------ box-plus */
int orc_constant(int frac_bits) { return (int)((5.0 / 8.0) * (1 << frac_bits)); } /* ArrayLDPCMacro.h:175 */

static inline int orc_sgn(int x) { return (x > 0) ? 1 : -1; }                     /* ArrayLDPCMacro.h:222-224 */

/* ArrayLDPC_Decoder.cpp:677-694 */
int orc_sxor(int x, int y, int C, int mask)
{
    int v1 = abs(x), v2 = abs(y);
    int sum = (v1 + v2) & mask;
    int diff = abs(v1 - v2) & mask;
    int part1 = C - (sum >> 2);
    part1 = part1 > 0 ? part1 : 0;
    int part2 = C - (diff >> 2);
    part2 = part2 > 0 ? part2 : 0;
    int mn = v1 < v2 ? v1 : v2;
    return orc_sgn(x) * orc_sgn(y) * (mn + part1 - part2);
}

void orc_sxor_table(int lo, int hi, int C, int mask, int32_t *out)
{
    int w = hi - lo + 1;
    for (int x = lo; x <= hi; x++)
        for (int y = lo; y <= hi; y++) out[(size_t)(x - lo) * w + (y - lo)] = orc_sxor(x, y, C, mask);
}

/* ------------------------------------------------------------------ syndrome */
/* checkPost_fp_general, ArrayLDPC_Decoder.cpp:296-333: hard = post > 0 ? 0 : 1, then XOR over
 * clist; 0 = pass. */
static int orc_check_post(const orc_code *H, const int32_t *post, uint8_t *hard)
{
    for (int v = 0; v < H->n; v++) hard[v] = post[v] > 0 ? 0 : 1;
    for (int c = 0; c < H->m; c++) {
        unsigned cs = 0;
        for (int k = 0; k < H->cdeg[c]; k++) cs ^= hard[H->clist[c * H->dc_max + k]];
        if (cs) return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------ decoder */
/* decode_general_fp, ArrayLDPC_Decoder.cpp:18-171.  Edge RAM: bank k, address c -> edge[k][c]
 * (ArrayLDPCMacro.h:85-106,162).  edge_io: the caller's edge RAM [dc_max][m] (FP_Decoder::EdgeRAM,
 * which outlives a call), or NULL for a per-call scratch; keep = 1 skips the edge init and iterates
 * from what edge_io holds (decode_fixpoint in state C2V, :462 / :488). */
int orc_decode_general_edges(const orc_code *H, const int32_t *llr, int max_iter, int C, int mask,
                             int32_t *edge_io, int keep, int32_t *post_out, uint8_t *hard_out, int *syn_ok)
{
    const int n = H->n, m = H->m, dc = H->dc_max, dv = H->dv_max;
    int *edge = edge_io ? edge_io : (int *)malloc(sizeof(int) * (size_t)dc * m); /* EdgeRAM[k].BRAM_fp[c] */
    int *addr_count = (int *)malloc(sizeof(int) * (size_t)m);
    int *mv2c = (int *)malloc(sizeof(int) * (size_t)dc);
    int *fwd = (int *)malloc(sizeof(int) * (size_t)dc);
    int *bwd = (int *)malloc(sizeof(int) * (size_t)dc);
    int *mc2v = (int *)malloc(sizeof(int) * (size_t)dv);
    int32_t *post = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    uint8_t *hard = (uint8_t *)malloc((size_t)n);
    int it, fail = 1;

    /* :45-61 edge init with channel values (skipped in state C2V, :462) */
    if (!keep)
        for (int c = 0; c < m; c++)
            for (int k = 0; k < H->cdeg[c]; k++) edge[k * m + c] = llr[H->clist[c * dc + k]];

    it = 0;
    while (it < max_iter) {
        /* :66-118 check-node phase, serial forward/backward fold per check */
        for (int c = 0; c < m; c++) {
            const int deg = H->cdeg[c];
            for (int k = 0; k < deg; k++) mv2c[k] = edge[k * m + c];
            fwd[0] = mv2c[0];
            bwd[deg - 1] = mv2c[deg - 1];
            for (int k = 1; k < deg; k++) {
                fwd[k] = orc_sxor(fwd[k - 1], mv2c[k], C, mask);
                bwd[deg - k - 1] = orc_sxor(bwd[deg - k], mv2c[deg - 1 - k], C, mask);
            }
            edge[0 * m + c] = bwd[1];
            edge[(deg - 1) * m + c] = fwd[deg - 2];
            for (int k = 1; k < deg - 1; k++) edge[k * m + c] = orc_sxor(fwd[k - 1], bwd[k + 1], C, mask);
        }
        /* :121-156 variable-node phase; bank = running addr_count[c] (relies on sorted rows) */
        for (int c = 0; c < m; c++) addr_count[c] = 0;
        for (int v = 0; v < n; v++) {
            int accum = 0;
            const int deg = H->vdeg[v];
            for (int k = 0; k < deg; k++) {
                const int c = H->vlist[v * dv + k];
                mc2v[k] = edge[addr_count[c] * m + c];
                accum += mc2v[k];
            }
            accum += llr[v];
            post[v] = accum;
            for (int k = 0; k < deg; k++) {
                const int c = H->vlist[v * dv + k];
                edge[addr_count[c] * m + c] = accum - mc2v[k];
                addr_count[c]++;
            }
        }
        it++;
        /* :164-167 early termination on the first passing syndrome */
        fail = orc_check_post(H, post, hard);
        if (!fail) break;
    }
    if (post_out) memcpy(post_out, post, sizeof(int32_t) * (size_t)n);
    if (hard_out) memcpy(hard_out, hard, (size_t)n);
    if (syn_ok) *syn_ok = !fail;
    if (!edge_io) free(edge);
    free(addr_count); free(mv2c); free(fwd); free(bwd); free(mc2v); free(post); free(hard);
    return it;
}

int orc_decode_general(const orc_code *H, const int32_t *llr, int max_iter, int C, int mask,
                       int32_t *post_out, uint8_t *hard_out, int *syn_ok)
{
    return orc_decode_general_edges(H, llr, max_iter, C, mask, NULL, 0, post_out, hard_out, syn_ok);
}

/* decode_fixpoint pre-check, hardDecision ArrayLDPC_Decoder.cpp:270-294 and :443-450.  For the
 * forward array code the ROM addressing (shift+j)%p + k*p equals clist, so the syndrome is taken
 * over clist here.  A passing pre-check returns before the edge RAM is touched. */
int orc_decode_fixpoint_edges(const orc_code *H, const int32_t *llr, int max_iter, int C, int mask,
                              int32_t *edge_io, int keep, int32_t *post, uint8_t *hard, int *syn_ok)
{
    uint8_t *hd = (uint8_t *)malloc((size_t)H->n);
    int fail = 0;
    for (int v = 0; v < H->n; v++) hd[v] = llr[v] > 0 ? 0 : 1;
    for (int c = 0; c < H->m && !fail; c++) {
        unsigned cs = 0;
        for (int k = 0; k < H->cdeg[c]; k++) cs ^= hd[H->clist[c * H->dc_max + k]];
        fail = cs != 0;
    }
    if (!fail) {
        if (hard) memcpy(hard, hd, (size_t)H->n);
        if (syn_ok) *syn_ok = 1;
        free(hd);
        return 0;
    }
    free(hd);
    return orc_decode_general_edges(H, llr, max_iter, C, mask, edge_io, keep, post, hard, syn_ok);
}

int orc_decode_fixpoint(const orc_code *H, const int32_t *llr, int max_iter, int C, int mask,
                        int32_t *post, uint8_t *hard, int *syn_ok)
{
    return orc_decode_fixpoint_edges(H, llr, max_iter, C, mask, NULL, 0, post, hard, syn_ok);
}

void orc_decode_batch(const orc_code *H, const void *llr, int llr_is_i16, int B, int max_iter,
                      int C, int mask, int precheck, int nthreads,
                      int32_t *iters, uint8_t *syn_ok, uint8_t *hard, int32_t *post)
{
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int f = 0; f < B; f++) {
        const size_t n = (size_t)H->n;
        int32_t *l32 = NULL;
        const int32_t *lp;
        if (llr_is_i16) {
            l32 = (int32_t *)malloc(sizeof(int32_t) * n);
            const int16_t *src = (const int16_t *)llr + (size_t)f * n;
            for (size_t i = 0; i < n; i++) l32[i] = src[i];
            lp = l32;
        } else {
            lp = (const int32_t *)llr + (size_t)f * n;
        }
        int ok = 0;
        int it = precheck
            ? orc_decode_fixpoint(H, lp, max_iter, C, mask, post ? post + f * n : NULL, hard ? hard + f * n : NULL, &ok)
            : orc_decode_general(H, lp, max_iter, C, mask, post ? post + f * n : NULL, hard ? hard + f * n : NULL, &ok);
        if (iters) iters[f] = it;
        if (syn_ok) syn_ok[f] = (uint8_t)ok;
        free(l32);
    }
}

/* ------------------------------------------------------------------ floating-point decoder */
/* FP_Decoder::sxor(double, double), ArrayLDPC_Decoder.cpp:724-732: exact Jacobian box-plus,
 * sgn(x)*sgn(y)*(min(|x|,|y|) + log(1 + exp(-(|x|+|y|))) - log(1 + exp(-||x|-|y||))), with
 * sgn(0) = -1 (ArrayLDPCMacro.h:218-220) and std::min (b < a ? b : a). */
double orc_sxor_f64(double x, double y)
{
    const double v1 = fabs(x), v2 = fabs(y);
    const double sum_abs = v1 + v2, diff_abs = fabs(v1 - v2);
    const double mn = (v2 < v1) ? v2 : v1;
    const int sg = ((x > 0) ? 1 : -1) * ((y > 0) ? 1 : -1);
    return sg * (mn + log(1 + exp(-sum_abs)) - log(1 + exp(-diff_abs)));
}

/* checkPost, ArrayLDPC_Decoder.cpp:335-372 (same rule as the fixed-point check on doubles). */
static int orc_check_post_f64(const orc_code *H, const double *post, uint8_t *hard)
{
    for (int v = 0; v < H->n; v++) hard[v] = post[v] > 0 ? 0 : 1;
    for (int c = 0; c < H->m; c++) {
        unsigned cs = 0;
        for (int k = 0; k < H->cdeg[c]; k++) cs ^= hard[H->clist[c * H->dc_max + k]];
        if (cs) return 1;
    }
    return 0;
}

/* FP_Decoder::decode_general(const double *LLR), ArrayLDPC_Decoder.cpp:735-933: the same
 * flooding schedule as decode_general_fp on doubles (EdgeRAM[k].BRAM[c], ArrayLDPCMacro.h:95-97):
 * edge init :762-778, check phase :782-835, variable phase :881-922 (accum = sum of c2v in vlist
 * order, THEN + LLR), early termination :926-929. */
int orc_decode_float(const orc_code *H, const double *llr, int max_iter, double *post_out,
                     uint8_t *hard_out, int *syn_ok)
{
    const int n = H->n, m = H->m, dc = H->dc_max, dv = H->dv_max;
    double *edge = (double *)malloc(sizeof(double) * (size_t)dc * m);
    int *addr_count = (int *)malloc(sizeof(int) * (size_t)m);
    double *mv2c = (double *)malloc(sizeof(double) * (size_t)dc);
    double *fwd = (double *)malloc(sizeof(double) * (size_t)dc);
    double *bwd = (double *)malloc(sizeof(double) * (size_t)dc);
    double *mc2v = (double *)malloc(sizeof(double) * (size_t)dv);
    double *post = (double *)malloc(sizeof(double) * (size_t)n);
    uint8_t *hard = (uint8_t *)malloc((size_t)n);
    int it = 0, fail = 1;

    for (int c = 0; c < m; c++)
        for (int k = 0; k < H->cdeg[c]; k++) edge[k * m + c] = llr[H->clist[c * dc + k]];
    while (it < max_iter) {
        for (int c = 0; c < m; c++) {
            const int deg = H->cdeg[c];
            for (int k = 0; k < deg; k++) mv2c[k] = edge[k * m + c];
            fwd[0] = mv2c[0];
            bwd[deg - 1] = mv2c[deg - 1];
            for (int k = 1; k < deg; k++) {
                fwd[k] = orc_sxor_f64(fwd[k - 1], mv2c[k]);
                bwd[deg - k - 1] = orc_sxor_f64(bwd[deg - k], mv2c[deg - 1 - k]);
            }
            edge[0 * m + c] = bwd[1];
            edge[(deg - 1) * m + c] = fwd[deg - 2];
            for (int k = 1; k < deg - 1; k++) edge[k * m + c] = orc_sxor_f64(fwd[k - 1], bwd[k + 1]);
        }
        for (int c = 0; c < m; c++) addr_count[c] = 0;
        for (int v = 0; v < n; v++) {
            double accum = 0;
            const int deg = H->vdeg[v];
            for (int k = 0; k < deg; k++) {
                const int c = H->vlist[v * dv + k];
                mc2v[k] = edge[addr_count[c] * m + c];
                accum = accum + mc2v[k];
            }
            accum = accum + llr[v];
            post[v] = accum;
            for (int k = 0; k < deg; k++) {
                const int c = H->vlist[v * dv + k];
                edge[addr_count[c] * m + c] = accum - mc2v[k];
                addr_count[c]++;
            }
        }
        it++;
        fail = orc_check_post_f64(H, post, hard);
        if (!fail) break;
    }
    if (post_out) memcpy(post_out, post, sizeof(double) * (size_t)n);
    if (hard_out) memcpy(hard_out, hard, (size_t)n);
    if (syn_ok) *syn_ok = !fail;
    free(edge); free(addr_count); free(mv2c); free(fwd); free(bwd); free(mc2v); free(post); free(hard);
    return it;
}

void orc_decode_float_batch(const orc_code *H, const double *llr, int B, int max_iter, int nthreads,
                            int32_t *iters, uint8_t *syn_ok, uint8_t *hard, double *post)
{
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int f = 0; f < B; f++) {
        const size_t n = (size_t)H->n;
        int ok = 0;
        const int it = orc_decode_float(H, llr + f * n, max_iter, post ? post + f * n : NULL,
                                        hard ? hard + f * n : NULL, &ok);
        if (iters) iters[f] = it;
        if (syn_ok) syn_ok[f] = (uint8_t)ok;
    }
}

/* ------------------------------------------------------------------ channel model */
#define ORC_MODULUS 2147483647LL /* rngs.cpp:40 */
#define ORC_MULT 48271LL         /* rngs.cpp:41 */

/* Random(), rngs.cpp:52-69 (Schrage's method; identical to the exact product mod m). */
double orc_random(int64_t *state)
{
    const int64_t Q = ORC_MODULUS / ORC_MULT, R = ORC_MODULUS % ORC_MULT;
    int64_t s = *state;
    int64_t t = ORC_MULT * (s % Q) - R * (s / Q);
    s = t > 0 ? t : t + ORC_MODULUS;
    *state = s;
    return (double)s / ORC_MODULUS;
}

/* Normal(m, s), rvgs.cpp:152-181: Odeh & Evans inverse CDF, one uniform per variate. */
double orc_normal(int64_t *state, double m, double s)
{
    const double p0 = 0.322232431088, q0 = 0.099348462606;
    const double p1 = 1.0, q1 = 0.588581570495;
    const double p2 = 0.342242088547, q2 = 0.531103462366;
    const double p3 = 0.204231210245e-1, q3 = 0.103537752850;
    const double p4 = 0.453642210148e-4, q4 = 0.385607006340e-2;
    double u, t, p, q, z;
    u = orc_random(state);
    if (u < 0.5) t = sqrt(-2.0 * log(u));
    else t = sqrt(-2.0 * log(1.0 - u));
    p = p0 + t * (p1 + t * (p2 + t * (p3 + t * p4)));
    q = q0 + t * (q1 + t * (q2 + t * (q3 + t * q4)));
    if (u < 0.5) z = (p / q) - t;
    else z = t - (p / q);
    return (m + s * z);
}

static int64_t orc_mulmod(int64_t a, int64_t b) { return (int64_t)(((__int128)a * b) % ORC_MODULUS); }

int64_t orc_skip(int64_t state, uint64_t k)
{
    int64_t r = 1, b = ORC_MULT;
    while (k) {
        if (k & 1) r = orc_mulmod(r, b);
        b = orc_mulmod(b, b);
        k >>= 1;
    }
    return orc_mulmod(state, r);
}

/* TestRandom, rngs.cpp:154-180 (first half: 10000 draws from seed 1 -> 399268537). */
int orc_test_random(void)
{
    int64_t s = 1;
    for (int i = 0; i < 10000; i++) orc_random(&s);
    return s == 399268537LL && orc_skip(1, 10000) == 399268537LL;
}

/* PerfTest.cpp:108-120 (WiFi harness) / :287-297 (array harness) / :168-169 (DecodeTrial). */
void orc_gen_llr(int64_t seed, int64_t f0, int B, int n, double snr, double sigma, int frac,
                 const uint8_t *cw, int32_t *out, int nthreads)
{
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int f = 0; f < B; f++) {
        int64_t s = orc_skip(seed, (uint64_t)(f0 + f) * (uint64_t)n);
        for (int i = 0; i < n; i++) {
            double llr = 2 * snr * (1 - 2 * (cw ? cw[i] : 0) + orc_normal(&s, 0, sigma));
            out[(size_t)f * n + i] = (int32_t)(llr * (1 << frac));
        }
    }
}

/* The unquantised LLR the float decoder takes: LLR = 2*snr*(1 - 2*cw[i] + Normal(0,sigma))
 * (PerfTest.cpp:108-110, before the int() of :111). */
void orc_gen_llr_f64(int64_t seed, int64_t f0, int B, int n, double snr, double sigma,
                     const uint8_t *cw, double *out, int nthreads)
{
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int f = 0; f < B; f++) {
        int64_t s = orc_skip(seed, (uint64_t)(f0 + f) * (uint64_t)n);
        for (int i = 0; i < n; i++)
            out[(size_t)f * n + i] = 2 * snr * (1 - 2 * (cw ? cw[i] : 0) + orc_normal(&s, 0, sigma));
    }
}

int orc_count_bit_errors(const uint8_t *hard, const int *info_index, const uint8_t *info_bits, int k)
{
    int e = 0;
    for (int i = 0; i < k; i++) e += hard[info_index[i]] != info_bits[i];
    return e;
}
