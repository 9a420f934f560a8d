// fpldpc_code.cpp -- parity-check code model: alist load/validate/write, native constructions
// (array codes, 802.11n n=1944 R=1/2), GF(2) rank and quasi-cyclic structure detection.
//
// Reference counterparts: FP_Decoder::ReadH (ArrayLDPC_Decoder.cpp:642-674), ROM
// (ArrayLDPCMacro.h:42-82), codes/alist_from_arraycode.m (array-code alist writer) and the data
// files H_array_p47_r5_forward.txt / H_802.11_IndZero.txt / codes/H_array_p47_r24_forward.txt,
// which tests/test_codes.py checks these constructions against token for token.
#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <numeric>
#include <sstream>

#include "fpldpc_internal.hpp"

namespace fpldpc {

static thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

// IEEE 802.11n-2009 rate-1/2, n = 1944, Z = 81 base matrix (shift, -1 = zero block); recovered
// from the reference's H_802.11_IndZero.txt, where check i*81+j connects var b*81+(j+s) mod 81.
static const int8_t kWifi1944R12[12][24] = {
    {57, -1, -1, -1, 50, -1, 11, -1, 50, -1, 79, -1, 1, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1},
    {3, -1, 28, -1, 0, -1, -1, -1, 55, 7, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1},
    {30, -1, -1, -1, 24, 37, -1, -1, 56, 14, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1},
    {62, 53, -1, -1, 53, -1, -1, 3, 35, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1},
    {40, -1, -1, 20, 66, -1, -1, 22, 28, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1},
    {0, -1, -1, -1, 8, -1, 42, -1, 50, -1, -1, 8, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1},
    {69, 79, 79, -1, -1, -1, 56, -1, 52, -1, -1, -1, 0, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1},
    {65, -1, -1, -1, 38, 57, -1, -1, 72, -1, 27, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1},
    {64, -1, -1, -1, 14, 52, -1, -1, 30, -1, -1, 32, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1},
    {-1, 45, -1, 70, 0, -1, -1, -1, 77, 9, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1},
    {2, 56, -1, 57, 35, -1, -1, -1, -1, -1, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0},
    {24, -1, 61, -1, 60, -1, -1, 27, 51, -1, -1, 16, 1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0},
};

static int gf2_rank(const fpldpc_code &c) {
    const int words = (c.n + 63) / 64;
    std::vector<uint64_t> rows((size_t)c.m * words, 0);
    for (int r = 0; r < c.m; r++)
        for (int k = 0; k < c.cdeg[r]; k++) {
            int v = c.clist[(size_t)r * c.dc_max + k];
            rows[(size_t)r * words + v / 64] ^= 1ull << (v % 64);
        }
    int rank = 0;
    for (int col = 0; col < c.n && rank < c.m; col++) {
        const int w = col / 64;
        const uint64_t bit = 1ull << (col % 64);
        int piv = -1;
        for (int r = rank; r < c.m; r++)
            if (rows[(size_t)r * words + w] & bit) { piv = r; break; }
        if (piv < 0) continue;
        if (piv != rank)
            for (int x = 0; x < words; x++) std::swap(rows[(size_t)piv * words + x], rows[(size_t)rank * words + x]);
        for (int r = 0; r < c.m; r++)
            if (r != rank && (rows[(size_t)r * words + w] & bit))
                for (int x = w; x < words; x++) rows[(size_t)r * words + x] ^= rows[(size_t)rank * words + x];
        rank++;
    }
    return rank;
}

// Largest Z dividing n and m for which every Z x Z block is zero or a cyclic shift of I.
static int detect_qc(const fpldpc_code &c) {
    int g = std::gcd(c.n, c.m);
    for (int z = g; z >= 2; z--) {
        if (g % z) continue;
        const int nb = c.n / z, mb = c.m / z;
        std::vector<int> shift((size_t)mb * nb, -1);
        bool ok = true;
        for (int cc = 0; cc < c.m && ok; cc++) {
            const int i = cc / z, j = cc % z;
            int cnt = 0;
            for (int k = 0; k < c.cdeg[cc] && ok; k++) {
                const int v = c.clist[(size_t)cc * c.dc_max + k];
                const int b = v / z, s = ((v % z) - j + z) % z;
                int &sh = shift[(size_t)i * nb + b];
                if (j == 0) {
                    if (sh != -1) ok = false;  // two ones in one block row of a block
                    sh = s;
                } else if (sh != s) {
                    ok = false;
                }
                cnt++;
            }
            if (ok && j > 0) {
                int expect = 0;
                for (int b = 0; b < nb; b++) expect += shift[(size_t)i * nb + b] >= 0;
                if (expect != cnt) ok = false;
            }
        }
        if (ok) return z;
    }
    return 0;
}

// Forward array code (codes/alist_from_arraycode.m, ROM::CirShift ArrayLDPCMacro.h:57): n = p^2,
// m = r*p, and slot k of check (i, j) is var k*p + (j + i*k) mod p.  Kernels use it to compute
// gather addresses instead of reading an index table.
static void detect_array(fpldpc_code *c) {
    c->array_forward = false;
    int p = 0;
    while (p * p < c->n) p++;
    if (p < 2 || p * p != c->n || c->m % p || c->dc_max != p) return;
    const int r = c->m / p;
    for (int i = 0; i < r; i++)
        for (int j = 0; j < p; j++) {
            const int row = i * p + j;
            if (c->cdeg[row] != p) return;
            for (int k = 0; k < p; k++)
                if (c->clist[(size_t)row * p + k] != k * p + (j + i * k) % p) return;
        }
    c->array_p = p;
    c->array_r = r;
    c->array_forward = true;
}

int code_finalize(fpldpc_code *c) {
    if (c->n <= 0 || c->m <= 0) return fail(FPLDPC_ERR_FORMAT, "alist: non-positive N or M");
    if (c->n > (1 << 16) - 1) return fail(FPLDPC_ERR_UNSUPPORTED, "code length above 65535");
    int64_t ev = 0, ec = 0;
    int dvm = 0, dcm = 0;
    for (int v = 0; v < c->n; v++) {
        const int d = c->vdeg[v];
        if (d < 0 || d > c->dv_max) return fail(FPLDPC_ERR_FORMAT, "alist: vdeg out of range at var " + std::to_string(v));
        ev += d;
        dvm = std::max(dvm, d);
        for (int k = 0; k < d; k++) {
            const int x = c->vlist[(size_t)v * c->dv_max + k];
            if (x < 0 || x >= c->m) return fail(FPLDPC_ERR_FORMAT, "alist: check index out of range in vlist row " + std::to_string(v));
            if (k && x <= c->vlist[(size_t)v * c->dv_max + k - 1])
                return fail(FPLDPC_ERR_FORMAT, "alist: vlist row " + std::to_string(v) + " not strictly ascending");
        }
    }
    for (int r = 0; r < c->m; r++) {
        const int d = c->cdeg[r];
        if (d < 0 || d > c->dc_max) return fail(FPLDPC_ERR_FORMAT, "alist: cdeg out of range at check " + std::to_string(r));
        ec += d;
        dcm = std::max(dcm, d);
        for (int k = 0; k < d; k++) {
            const int x = c->clist[(size_t)r * c->dc_max + k];
            if (x < 0 || x >= c->n) return fail(FPLDPC_ERR_FORMAT, "alist: var index out of range in clist row " + std::to_string(r));
            // The reference selects the edge bank of (c, v) by counting vars of c in ascending
            // order (addr_count, ArrayLDPC_Decoder.cpp:137), i.e. it assumes sorted clist rows.
            if (k && x <= c->clist[(size_t)r * c->dc_max + k - 1])
                return fail(FPLDPC_ERR_FORMAT, "alist: clist row " + std::to_string(r) + " not strictly ascending");
        }
    }
    if (ev != ec) return fail(FPLDPC_ERR_FORMAT, "alist: sum(vdeg) != sum(cdeg)");
    // vlist/clist consistency: every (v, c) in vlist appears in clist.
    for (int v = 0; v < c->n; v++)
        for (int k = 0; k < c->vdeg[v]; k++) {
            const int r = c->vlist[(size_t)v * c->dv_max + k];
            const int32_t *row = &c->clist[(size_t)r * c->dc_max];
            if (!std::binary_search(row, row + c->cdeg[r], v))
                return fail(FPLDPC_ERR_FORMAT, "alist: vlist/clist mismatch at var " + std::to_string(v));
        }
    c->edges = ec;
    c->regular_checks = true;
    for (int r = 0; r < c->m; r++) c->regular_checks &= c->cdeg[r] == c->dc_max;
    c->rank = gf2_rank(*c);
    c->qc_z = detect_qc(*c);
    detect_array(c);
    (void)dvm;
    (void)dcm;
    return FPLDPC_OK;
}

static int parse_ints(const char *text, size_t len, std::vector<long> *out) {
    const char *p = text, *end = text + len;
    while (p < end) {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
        if (p >= end) break;
        char *q = nullptr;
        errno = 0;
        long x = strtol(p, &q, 10);
        if (q == p || errno) return fail(FPLDPC_ERR_FORMAT, "alist: non-integer token");
        out->push_back(x);
        p = q;
    }
    return FPLDPC_OK;
}

static int build_from_tokens(const std::vector<long> &t, fpldpc_code *c) {
    size_t i = 0;
    auto next = [&](long *x) -> bool {
        if (i >= t.size()) return false;
        *x = t[i++];
        return true;
    };
    long n, m, dv, dc;
    if (!next(&n) || !next(&m) || !next(&dv) || !next(&dc)) return fail(FPLDPC_ERR_FORMAT, "alist: truncated header");
    if (n <= 0 || m <= 0 || dv <= 0 || dc <= 0 || n > 1000000 || m > 1000000 || dv > 4096 || dc > 4096)
        return fail(FPLDPC_ERR_FORMAT, "alist: bad header");
    c->n = (int)n;
    c->m = (int)m;
    c->dv_max = (int)dv;
    c->dc_max = (int)dc;
    c->vdeg.assign(n, 0);
    c->cdeg.assign(m, 0);
    c->vlist.assign((size_t)n * dv, -1);
    c->clist.assign((size_t)m * dc, -1);
    long x;
    for (long v = 0; v < n; v++) {
        if (!next(&x) || x < 0 || x > dv) return fail(FPLDPC_ERR_FORMAT, "alist: bad vdeg");
        c->vdeg[v] = (int)x;
    }
    for (long r = 0; r < m; r++) {
        if (!next(&x) || x < 0 || x > dc) return fail(FPLDPC_ERR_FORMAT, "alist: bad cdeg");
        c->cdeg[r] = (int)x;
    }
    for (long v = 0; v < n; v++)
        for (int k = 0; k < c->vdeg[v]; k++) {
            if (!next(&x)) return fail(FPLDPC_ERR_FORMAT, "alist: truncated vlist");
            c->vlist[(size_t)v * dv + k] = (int)x;
        }
    for (long r = 0; r < m; r++)
        for (int k = 0; k < c->cdeg[r]; k++) {
            if (!next(&x)) return fail(FPLDPC_ERR_FORMAT, "alist: truncated clist");
            c->clist[(size_t)r * dc + k] = (int)x;
        }
    if (i != t.size()) return fail(FPLDPC_ERR_FORMAT, "alist: trailing tokens");
    return code_finalize(c);
}

// Builds vlist from clist (ascending by construction when checks are visited in order).
static void fill_vlist(fpldpc_code *c) {
    c->vdeg.assign(c->n, 0);
    for (int r = 0; r < c->m; r++)
        for (int k = 0; k < c->cdeg[r]; k++) c->vdeg[c->clist[(size_t)r * c->dc_max + k]]++;
    c->dv_max = *std::max_element(c->vdeg.begin(), c->vdeg.end());
    c->vlist.assign((size_t)c->n * c->dv_max, -1);
    std::vector<int> fill(c->n, 0);
    for (int r = 0; r < c->m; r++)
        for (int k = 0; k < c->cdeg[r]; k++) {
            const int v = c->clist[(size_t)r * c->dc_max + k];
            c->vlist[(size_t)v * c->dv_max + fill[v]++] = r;
        }
}

}  // namespace fpldpc

using namespace fpldpc;

extern "C" {

const char *fpldpc_last_error(void) { return g_last_error.c_str(); }
const char *fpldpc_version(void) { return "fpldpc 0.1 (gfx950)"; }

#ifndef FPLDPC_KERNEL_BUILD_ID
#define FPLDPC_KERNEL_BUILD_ID "unknown"
#endif
const char *fpldpc_kernel_build_id(void) { return FPLDPC_KERNEL_BUILD_ID; }

int fpldpc_code_parse_alist(const char *text, size_t len, fpldpc_code_t *out) {
    if (!text || !out) return fail(FPLDPC_ERR_ARG, "null argument");
    std::vector<long> toks;
    int st = parse_ints(text, len, &toks);
    if (st) return st;
    std::unique_ptr<fpldpc_code> c(new fpldpc_code());
    st = build_from_tokens(toks, c.get());
    if (st) return st;
    *out = c.release();
    return FPLDPC_OK;
}

int fpldpc_code_load_alist(const char *path, fpldpc_code_t *out) {
    if (!path || !out) return fail(FPLDPC_ERR_ARG, "null argument");
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(FPLDPC_ERR_IO, std::string("cannot open ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    std::string s = ss.str();
    return fpldpc_code_parse_alist(s.data(), s.size(), out);
}

int fpldpc_code_array(int32_t p, int32_t r, int32_t forward, fpldpc_code_t *out) {
    if (!out || p < 2 || r < 1 || r > p || p > 255) return fail(FPLDPC_ERR_ARG, "array code needs 2 <= p <= 255, 1 <= r <= p");
    for (int d = 2; d * d <= p; d++)
        if (p % d == 0) return fail(FPLDPC_ERR_ARG, "array code needs p prime");
    std::unique_ptr<fpldpc_code> c(new fpldpc_code());
    c->n = p * p;
    c->m = r * p;
    c->dc_max = p;
    c->cdeg.assign(c->m, p);
    c->clist.assign((size_t)c->m * p, -1);
    for (int i = 0; i < r; i++)
        for (int j = 0; j < p; j++)
            for (int k = 0; k < p; k++) {
                // ROM::CirShift[i][k] = (i*k) mod p (ArrayLDPCMacro.h:57); var group k.
                const int s = (i * k) % p;
                const int col = forward ? (j + s) % p : ((j - s) % p + p) % p;
                c->clist[((size_t)i * p + j) * p + k] = k * p + col;
            }
    fill_vlist(c.get());
    c->array_p = p;
    c->array_r = r;
    int st = code_finalize(c.get());
    if (st) return st;
    *out = c.release();
    return FPLDPC_OK;
}

int fpldpc_code_wifi_1944_r12(fpldpc_code_t *out) {
    if (!out) return fail(FPLDPC_ERR_ARG, "null argument");
    const int Z = 81;
    std::unique_ptr<fpldpc_code> c(new fpldpc_code());
    c->n = 24 * Z;
    c->m = 12 * Z;
    c->dc_max = 8;
    c->cdeg.assign(c->m, 0);
    c->clist.assign((size_t)c->m * c->dc_max, -1);
    for (int i = 0; i < 12; i++)
        for (int j = 0; j < Z; j++) {
            const int r = i * Z + j;
            int d = 0;
            for (int b = 0; b < 24; b++)
                if (kWifi1944R12[i][b] >= 0) c->clist[(size_t)r * c->dc_max + d++] = b * Z + (j + kWifi1944R12[i][b]) % Z;
            c->cdeg[r] = d;
        }
    fill_vlist(c.get());
    int st = code_finalize(c.get());
    if (st) return st;
    *out = c.release();
    return FPLDPC_OK;
}

int fpldpc_code_dims(fpldpc_code_t c, int32_t dims[8]) {
    if (!c || !dims) return fail(FPLDPC_ERR_ARG, "null argument");
    dims[0] = c->n;
    dims[1] = c->m;
    dims[2] = c->dv_max;
    dims[3] = c->dc_max;
    dims[4] = (int32_t)c->edges;
    dims[5] = c->qc_z;
    dims[6] = c->rank;
    dims[7] = c->regular_checks ? 1 : 0;
    return FPLDPC_OK;
}

int fpldpc_code_rate(fpldpc_code_t c, double *rate) {
    if (!c || !rate) return fail(FPLDPC_ERR_ARG, "null argument");
    if (c->array_p) {
        const int P = c->array_p, R = c->array_r;
        *rate = 1 - double(R * P - R + 1) / (P * P);  // ROM::CodeRate, ArrayLDPCMacro.h:60
    } else {
        *rate = 1 - double(c->rank) / c->n;
    }
    return FPLDPC_OK;
}

int fpldpc_code_lists(fpldpc_code_t c, int32_t *vdeg, int32_t *cdeg, int32_t *vlist, int32_t *clist) {
    if (!c) return fail(FPLDPC_ERR_ARG, "null argument");
    if (vdeg) memcpy(vdeg, c->vdeg.data(), sizeof(int32_t) * c->n);
    if (cdeg) memcpy(cdeg, c->cdeg.data(), sizeof(int32_t) * c->m);
    if (vlist) memcpy(vlist, c->vlist.data(), sizeof(int32_t) * c->vlist.size());
    if (clist) memcpy(clist, c->clist.data(), sizeof(int32_t) * c->clist.size());
    return FPLDPC_OK;
}

int fpldpc_code_write_alist(fpldpc_code_t c, char *buf, size_t cap, size_t *len) {
    if (!c || !len) return fail(FPLDPC_ERR_ARG, "null argument");
    std::ostringstream o;
    o << c->n << " " << c->m << "\n" << c->dv_max << " " << c->dc_max << "\n";
    for (int v = 0; v < c->n; v++) o << c->vdeg[v] << (v + 1 < c->n ? " " : "\n");
    for (int r = 0; r < c->m; r++) o << c->cdeg[r] << (r + 1 < c->m ? " " : "\n");
    for (int v = 0; v < c->n; v++) {
        for (int k = 0; k < c->vdeg[v]; k++) o << c->vlist[(size_t)v * c->dv_max + k] << " ";
        o << "\n";
    }
    for (int r = 0; r < c->m; r++) {
        for (int k = 0; k < c->cdeg[r]; k++) o << c->clist[(size_t)r * c->dc_max + k] << " ";
        o << "\n";
    }
    const std::string s = o.str();
    *len = s.size();
    if (buf && cap > 0) {
        const size_t w = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), w);
        buf[w] = 0;
    }
    return FPLDPC_OK;
}

int fpldpc_code_syndrome_host(fpldpc_code_t c, const uint8_t *bits) {
    if (!c || !bits) return fail(FPLDPC_ERR_ARG, "null argument");
    for (int r = 0; r < c->m; r++) {
        unsigned x = 0;
        for (int k = 0; k < c->cdeg[r]; k++) x ^= bits[c->clist[(size_t)r * c->dc_max + k]] & 1u;
        if (x) return 1;
    }
    return 0;
}

void fpldpc_code_free(fpldpc_code_t c) { delete c; }

}  // extern "C"
