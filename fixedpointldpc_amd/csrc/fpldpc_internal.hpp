// fpldpc_internal.hpp -- host-side internals shared by the libfpldpc.so translation units.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "fpldpc.h"

// Parity-check code in alist form (0-based, rows ascending), the data the reference keeps in
// FP_Decoder::{vnum, cnum, vdeg, cdeg, vlist, clist} (ArrayLDPCMacro.h:171-172).
struct fpldpc_code {
    int n = 0, m = 0, dv_max = 0, dc_max = 0;
    int64_t edges = 0;
    std::vector<int32_t> vdeg, cdeg;
    std::vector<int32_t> vlist;  // [n][dv_max], -1 padded
    std::vector<int32_t> clist;  // [m][dc_max], -1 padded; clist order = fold order
    int qc_z = 0;                // circulant size if quasi-cyclic, else 0
    int rank = -1;               // GF(2) rank of H
    bool regular_checks = false; // every check has degree dc_max
    int array_p = 0, array_r = 0;// array code p x r (built by fpldpc_code_array or detected)
    bool array_forward = false;  // check (i,j) slot k -> var k*p + (j + i*k) mod p
};

namespace fpldpc {

// Thread-local last-error plumbing for the C ABI.
int fail(int code, const std::string &msg);
int fail_hip(int hip_status, const char *what);

int code_finalize(fpldpc_code *c);  // validate + derived fields; returns status

// HIP kernel launch front-end (fpldpc_kernels.hip).
struct DeviceCode {
    int n = 0, m = 0, dc = 0;         // dc = kernel DC (>= code dc_max)
    int m_pad = 0;                    // row pitch of vidx
    const uint16_t *vidx = nullptr;   // [dc][m_pad] var index of slot k of check c
    const uint8_t *cdeg = nullptr;    // [m]
};

struct LaunchArgs {
    const void *llr = nullptr;
    int llr_i16 = 0;
    int batch = 0;
    int max_iter = 30, C = 10, mask = 0xff, early_term = 1, precheck = 0;
    uint32_t *hard = nullptr;
    int hard_words = 0;
    int32_t *iters = nullptr;
    uint8_t *syn_ok = nullptr;
    int32_t *post = nullptr;
    int32_t *bit_errors = nullptr;
    unsigned long long *totals = nullptr;
    const int32_t *info_idx = nullptr;
    const uint8_t *info_bits = nullptr;
    int k_info = 0;
    const uint32_t *info_mask = nullptr;  // [2][hard_words] info positions / reference bits, or null
    int *work_counter = nullptr;   // the decoder's counter block (kCounterInts), zero between calls
    int32_t *c2v_scratch = nullptr;// [grid][dc][m_pad] for the global-memory variant
    uint32_t bfe_w = 6;            // width_mask = 2^(bfe_w+2) - 1
    int *fb_list = nullptr;        // [lists][batch] frames handed down the fallback chain (packed variants)
    unsigned long long *probe = nullptr;  // diagnostic clock probe (host-mapped), or null
    unsigned long long *wgtrace = nullptr;  // diagnostic per-workgroup trace [grid][4] (host-mapped), or null
    int split_tail = 1;            // packed array kernels: a lone frame continues in the split form
};

enum class Variant { kNone, kArray47x2, kArray47x2c2, kArray47x2c2t, kArray47x2mix, kArray47, kLds16_47, kTab8x4lo3, kTab8x4p, kReg47x1Regular, kReg8x4, kReg8x1, kReg16x2, kGmem8, kGmem16, kGmem32, kGmem48, kGmem64 };

struct KernelChoice {
    Variant v = Variant::kNone;
    int threads = 256;
    int grid = 0;            // resident workgroups (persistent)
    size_t lds_bytes = 0;
    size_t scratch_ints = 0; // c2v scratch per launch (global variant)
    const char *name = "";
    Variant fallback = Variant::kNone;  // packed kernels: int32 re-decode of out-of-range frames
    int fb_grid = 0, fb_threads = 0;
    size_t fb_lds = 0;
    uint32_t cmax = 0;
    Variant fallback2 = Variant::kNone;  // the fallback's own fallback (a chain of at most 3 kernels)
    int fb2_grid = 0, fb2_threads = 0;
    size_t fb2_lds = 0;
    bool sort_checks = false;  // the var-index table lists the checks by ascending degree (stable)
    int lists() const { return fallback == Variant::kNone ? 0 : fallback2 == Variant::kNone ? 1 : 2; }
};

// Per-decoder device counter block (int32): [0] work counter, [1] first fallback's work counter,
// [2] frames in fallback list 0, [3] second fallback's work counter, [4] frames in list 1,
// [5] workgroups out of the call's last kernel, [6] / [7] the last call's list 0 / 1 sizes.
// Zeroed once at decoder creation; the last workgroup of each call's last kernel resets [0..5]
// (chain_exit, fpldpc_kernels.hip), so a decode call issues kernels only.
constexpr int kCounterInts = 8;
constexpr int kCountFb0 = 2;
constexpr int kCountFb1 = 4;
constexpr int kCountExit = 5;
constexpr int kCountFb0Last = 6;
constexpr int kCountFb1Last = 7;

// Kernel DC (slot rows of the vidx table) of a variant.
int kernel_dc(Variant v);
// Picks a variant for the code, WIDTH_MASK and Constant C and the device; fills grid from the
// occupancy query.
int choose_kernel(const fpldpc_code &code, int device, int mask, int C, KernelChoice *out);
// Launches on stream (hipStream_t).  The counter block must be zero (it is between calls).
int launch_decode(const KernelChoice &kc, const DeviceCode &dcode, const LaunchArgs &args, void *stream);
// A second decoder of src's code, parameters, device and resolved kernel choice (not re-read from the
// environment), diagnostics off: fpldpc_ber_sim's second chunk in flight.
int decoder_create_twin(fpldpc_decoder_t src, fpldpc_decoder_t *out);

// The stateful single-frame decode (fpldpc_decode_frame): its own index table in the code's check
// order, built on first use.  vidx [dc_max][m] (slot k of check c), c2v [2][dc][m] scratch.
struct EdgeTables {
    int n = 0, m = 0, dc = 0;  // dc = edge_kernel_dc(dc_max)
    int dc_max = 0;            // rows of vidx ([dc_max][m])
    uint16_t *vidx = nullptr;
    uint8_t *cdeg = nullptr;
    int32_t *c2v = nullptr;
};
int edge_kernel_dc(int dc_max);  // 8 / 16 / 32 / 48 / 64, 0 if dc_max > 64
// One frame on stream: edge [dc_max][m] device edge RAM, in/out (fpldpc_kernels.hip flood_edges).
int launch_decode_frame(const LaunchArgs &args, const EdgeTables &t, int32_t *edge, int keep, void *stream);

}  // namespace fpldpc

namespace fpldpc {
struct FloatState;  // floating-point decoder tables (fpldpc_float.hip), built on first use
void free_float_state(FloatState *s);
}  // namespace fpldpc

// Decoder object (fpldpc_decoder_t): device-resident code description + kernel choice.
struct fpldpc_decoder {
    fpldpc_code code;
    fpldpc_params params{};
    int device = 0;
    fpldpc::KernelChoice kc;
    fpldpc::DeviceCode dcode;
    uint16_t *d_vidx = nullptr;
    uint8_t *d_cdeg = nullptr;
    int *d_counter = nullptr;
    int32_t *d_scratch = nullptr;
    unsigned long long *h_probe = nullptr;  // FPLDPC_CLOCK_PROBE diagnostic (host-mapped)
    unsigned long long *h_wgtrace = nullptr;  // FPLDPC_WG_TRACE diagnostic (host-mapped, [grid][4])
    int *d_fb_list = nullptr;      // fallback frame list of the packed kernels
    bool diag_probe = false;        // FPLDPC_CLOCK_PROBE=1 at creation
    bool split_tail = true;         // FPLDPC_SPLIT_TAIL=0 at creation: no split form in the tail (A/B runs)
    std::string diag_trace_path;    // FPLDPC_WG_TRACE at creation
    int fb_cap = 0;
    int32_t *d_info_idx = nullptr;
    uint8_t *d_info_bits = nullptr;
    uint32_t *d_info_mask = nullptr;  // packed [2][hard words] when the info positions are distinct
    int k_info = 0;
    // staging for fpldpc_decode_host
    hipStream_t stream = nullptr;
    hipEvent_t last_done = nullptr;  // recorded after each (uncaptured) decode: fallback_counts waits on it
    void *d_stage = nullptr;
    size_t stage_bytes = 0;
    fpldpc::FloatState *fl = nullptr;
    fpldpc::EdgeTables edges;        // fpldpc_decode_frame tables (first use)
    int32_t *d_edge_stage = nullptr; // fpldpc_decode_frame_host staging: llr, edge RAM, post, hard, iters, ok
    int32_t *h_edge_stage = nullptr; // the same block in pinned host memory (one copy each way per call)
};

// Systematic encoder (fpldpc_encoder_t), host tables + lazily uploaded device tables.
struct fpldpc_encoder {
    int n = 0, k = 0;
    std::vector<int32_t> info_index;    // [k] ascending (getInfoIndex)
    std::vector<int32_t> parity_index;  // [n-k]
    std::vector<int32_t> row_ptr;       // CSR over parity rows: info VAR indices XORed into parity r
    std::vector<int32_t> row_var;
    std::vector<int32_t> info_slot;     // var -> slot in info_index, -1 for parity vars
    // device side (fpldpc_encoder_encode): per codeword position v, its info slot (>= 0) or
    // -(r + 1) for parity row r; row masks over info slots [n-k][kw] bit-packed
    int device = -1, kw = 0;
    int32_t *d_pos = nullptr;
    uint32_t *d_rowmask = nullptr;
    uint32_t *d_packed = nullptr;  // scratch: packed info bits [cap][kw]
    int cap = 0;
    ~fpldpc_encoder();
};

namespace fpldpc {
// device-side encoder / channel launchers (fpldpc_gen.hip)
int encoder_upload(fpldpc_encoder *e);
int launch_encode(fpldpc_encoder *e, const uint8_t *info, int batch, uint8_t *cw, void *stream);
int launch_channel(int64_t seed, int64_t first_frame, int frames, int n, double snr, double sigma, int frac_bits,
                   const uint8_t *cw, int cw_per_frame, void *out, int out_type, int *overflow, void *stream);
// llr[f][idx[i]] = value for every frame (the harness's shortening, PerfTest.cpp:410-414)
int launch_force_llr(int16_t *llr, int frames, int n, const int32_t *idx, int n_idx, int16_t value, void *stream);
}  // namespace fpldpc
