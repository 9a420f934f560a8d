// fpldpc_encoder.cpp -- systematic encoder (host): the reference's G-file encoder and a native
// one derived from H.
//
// Reference: FP_Encoder (ArrayLDPC_Encoder.cpp:34-157 reads "N M_G / x cmax / ColumnFlag[N] /
// ChkDeg[M_G] / rows", :160-225 encodes: info bits at the ColumnFlag == 0 positions in ascending
// order, parity i = XOR of the info bits listed in G row i).  The G files were made offline by
// codes/simplfy_generator_alist.m from a Gaussian-eliminated H; fpldpc_encoder_from_code makes
// the same object natively: parity positions = the pivot columns of a column-order GF(2) row
// reduction of H, parity row = the free columns of that pivot's reduced row.  tests/test_encoder.py
// checks both against the reference's KAT codewords.
#include <algorithm>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <thread>

#include "fpldpc_internal.hpp"

using namespace fpldpc;

// Device tables exist only once fpldpc_encoder_encode has run (a host-only encoder makes no HIP call).
fpldpc_encoder::~fpldpc_encoder() {
    if (d_pos) (void)hipFree(d_pos);
    if (d_rowmask) (void)hipFree(d_rowmask);
    if (d_packed) (void)hipFree(d_packed);
}

namespace {

int finish(std::unique_ptr<fpldpc_encoder> &e, fpldpc_encoder_t *out) {
    e->info_slot.assign(e->n, -1);
    for (int i = 0; i < e->k; i++) e->info_slot[e->info_index[i]] = i;
    for (int32_t v : e->row_var)
        if (v < 0 || v >= e->n || e->info_slot[v] < 0)
            return fail(FPLDPC_ERR_FORMAT, "encoder row references a non-information position");
    *out = e.release();
    return FPLDPC_OK;
}

}  // namespace

extern "C" {

int fpldpc_encoder_load_g(const char *path, fpldpc_encoder_t *out) {
    if (!path || !out) return fail(FPLDPC_ERR_ARG, "null argument");
    std::ifstream f(path);
    if (!f) return fail(FPLDPC_ERR_IO, std::string("cannot open ") + path);
    long n, mg, x, cmax;
    if (!(f >> n >> mg >> x >> cmax) || n <= 0 || mg <= 0 || mg >= n || n > 1000000)
        return fail(FPLDPC_ERR_FORMAT, "G file: bad header");
    std::unique_ptr<fpldpc_encoder> e(new fpldpc_encoder());
    e->n = (int)n;
    std::vector<int> flag(n);
    for (long i = 0; i < n; i++) {
        if (!(f >> flag[i]) || (flag[i] != 0 && flag[i] != 1)) return fail(FPLDPC_ERR_FORMAT, "G file: bad ColumnFlag");
        (flag[i] ? e->parity_index : e->info_index).push_back((int32_t)i);
    }
    if ((long)e->parity_index.size() != mg) return fail(FPLDPC_ERR_FORMAT, "G file: ColumnFlag count != M_G");
    e->k = (int)e->info_index.size();
    std::vector<long> deg(mg);
    for (long r = 0; r < mg; r++)
        if (!(f >> deg[r]) || deg[r] < 0 || deg[r] > n) return fail(FPLDPC_ERR_FORMAT, "G file: bad row degree");
    e->row_ptr.push_back(0);
    for (long r = 0; r < mg; r++) {
        for (long j = 0; j < deg[r]; j++) {
            long v;
            if (!(f >> v) || v < 0 || v >= n) return fail(FPLDPC_ERR_FORMAT, "G file: bad row entry");
            // encode() skips parity columns listed in a row (ColumnFlag test, :213-218)
            if (!flag[v]) e->row_var.push_back((int32_t)v);
        }
        e->row_ptr.push_back((int32_t)e->row_var.size());
    }
    return finish(e, out);
}

int fpldpc_encoder_from_code(fpldpc_code_t code, fpldpc_encoder_t *out) {
    if (!code || !out) return fail(FPLDPC_ERR_ARG, "null argument");
    const int n = code->n, m = code->m, W = (n + 63) / 64;
    std::vector<uint64_t> rows((size_t)m * W, 0);
    for (int r = 0; r < m; r++)
        for (int j = 0; j < code->cdeg[r]; j++) {
            const int v = code->clist[(size_t)r * code->dc_max + j];
            rows[(size_t)r * W + v / 64] ^= 1ull << (v % 64);
        }
    // Gauss-Jordan over GF(2), pivots taken in ascending column order.
    std::vector<int> pivot_col;
    int rank = 0;
    for (int col = 0; col < n && rank < m; col++) {
        const int w = col / 64;
        const uint64_t bit = 1ull << (col % 64);
        int piv = -1;
        for (int r = rank; r < m; r++)
            if (rows[(size_t)r * W + w] & bit) {
                piv = r;
                break;
            }
        if (piv < 0) continue;
        if (piv != rank)
            for (int x = 0; x < W; x++) std::swap(rows[(size_t)piv * W + x], rows[(size_t)rank * W + x]);
        for (int r = 0; r < m; r++)
            if (r != rank && (rows[(size_t)r * W + w] & bit))
                for (int x = 0; x < W; x++) rows[(size_t)r * W + x] ^= rows[(size_t)rank * W + x];
        pivot_col.push_back(col);
        rank++;
    }
    std::unique_ptr<fpldpc_encoder> e(new fpldpc_encoder());
    e->n = n;
    std::vector<char> is_piv(n, 0);
    for (int c : pivot_col) is_piv[c] = 1;
    for (int v = 0; v < n; v++) (is_piv[v] ? e->parity_index : e->info_index).push_back(v);
    e->k = (int)e->info_index.size();
    e->row_ptr.push_back(0);
    for (int r = 0; r < rank; r++) {
        for (int v = 0; v < n; v++)
            if (!is_piv[v] && (rows[(size_t)r * W + v / 64] >> (v % 64) & 1)) e->row_var.push_back(v);
        e->row_ptr.push_back((int32_t)e->row_var.size());
    }
    return finish(e, out);
}

int fpldpc_encoder_dims(fpldpc_encoder_t e, int32_t dims[3]) {
    if (!e || !dims) return fail(FPLDPC_ERR_ARG, "null argument");
    dims[0] = e->n;
    dims[1] = e->k;
    int mx = 0;
    for (size_t r = 0; r + 1 < e->row_ptr.size(); r++) mx = std::max(mx, e->row_ptr[r + 1] - e->row_ptr[r]);
    dims[2] = mx;
    return FPLDPC_OK;
}

int fpldpc_encoder_info_index(fpldpc_encoder_t e, int32_t *info_index, int32_t *parity_index) {
    if (!e) return fail(FPLDPC_ERR_ARG, "null argument");
    if (info_index) memcpy(info_index, e->info_index.data(), sizeof(int32_t) * e->k);
    if (parity_index) memcpy(parity_index, e->parity_index.data(), sizeof(int32_t) * e->parity_index.size());
    return FPLDPC_OK;
}

int fpldpc_unpack_info_bytes(const char *in, int32_t in_len, int32_t k, uint8_t *bits) {
    // FP_Decoder::setInfoBit (ArrayLDPC_Decoder.cpp:178-197) == FP_Encoder::encode's unpacking
    // (ArrayLDPC_Encoder.cpp:181-196): LSB first, bytes 0..in_len-2 whole, then k % 8 bits of the
    // last byte.  Bits beyond what the bytes supply are 0.
    if (!in || !bits || in_len < 1 || k < 0) return fail(FPLDPC_ERR_ARG, "bad argument");
    memset(bits, 0, (size_t)k);
    int c = 0;
    for (int i = 0; i < in_len - 1; i++)
        for (int j = 0; j < 8; j++, c++)
            if (c < k) bits[c] = (uint8_t)((in[i] >> j) & 1);
    for (int j = 0; j < k % 8; j++, c++)
        if (c < k) bits[c] = (uint8_t)((in[in_len - 1] >> j) & 1);
    return FPLDPC_OK;
}

int fpldpc_encoder_encode_host(fpldpc_encoder_t e, const uint8_t *info, int32_t batch, uint8_t *cw, int32_t nthreads) {
    if (!e || !info || !cw || batch < 0) return fail(FPLDPC_ERR_ARG, "bad argument");
    const int n = e->n, k = e->k, R = (int)e->row_ptr.size() - 1;
    auto work = [&](int64_t lo, int64_t hi) {
        for (int64_t b = lo; b < hi; b++) {
            const uint8_t *u = info + (size_t)b * k;
            uint8_t *c = cw + (size_t)b * n;
            for (int i = 0; i < k; i++) c[e->info_index[i]] = u[i] & 1;  // encode(), :197-200
            for (int r = 0; r < R; r++) {                                  // :211-223
                uint8_t x = 0;
                for (int j = e->row_ptr[r]; j < e->row_ptr[r + 1]; j++) x ^= c[e->row_var[j]];
                c[e->parity_index[r]] = x;
            }
        }
    };
    unsigned hw = std::thread::hardware_concurrency();
    int T = nthreads > 0 ? nthreads : (int)(hw ? hw : 1);
    T = std::max(1, std::min<int>(T, batch));
    if (T == 1) {
        work(0, batch);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) th.emplace_back(work, (int64_t)batch * t / T, (int64_t)batch * (t + 1) / T);
        for (auto &x : th) x.join();
    }
    return FPLDPC_OK;
}

void fpldpc_encoder_free(fpldpc_encoder_t e) { delete e; }

}  // extern "C"
