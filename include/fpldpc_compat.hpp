// fpldpc_compat.hpp -- the reference's C++ API (tyc85/FixedPointLDPC) on top of libfpldpc.so.
//
// Drop-in for code written against ArrayLDPCMacro.h / PerfTest.h: the same class names, member
// functions, argument meanings and return values, with the decode running on the MI355X.
//   FP_Decoder   ArrayLDPCMacro.h:121-176   (decode_general_fp, decode_fixpoint, decode_general,
//                                            ReadH, getPost_fp, getPost, setState, setInfoBit,
//                                            setInfoIndex, calculateBER, checkPost, sxor, ...)
//   FP_Encoder   ArrayLDPCMacro.h:179-214   (FP_Encoder(char*, int), encode (both overloads),
//                                            getCodeword, getInfoIndex)
//   PerfTest.h   PerfTest.h:4-11            (ArrayLDPC_Debug, ArrayLDPC_Debug_Wifi, DecodeTrial, ...)
// Differences, all deliberate:
//   * errors throw fpldpc_error (the reference exits, or silently continues with zeroed arrays);
//   * ReadH takes an optional path (the reference hard-codes "H_802.11_IndZero.txt",
//     ArrayLDPC_Decoder.cpp:646 -- still the default);
//   * decoder state is per object (no function statics, ArrayLDPC_Decoder.cpp:21-37);
//   * decode_batch() is added: the per-frame calls cost one GPU round trip each, the batch call is
//     the fast path (fpldpc_decode).  It neither reads nor writes the edge RAM or the FSM state:
//     those belong to the per-frame calls (fpldpc_decode_frame).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "fpldpc.h"

struct fpldpc_error : std::runtime_error {
    int code;
    fpldpc_error(int c, const std::string &what) : std::runtime_error(what), code(c) {}
};

namespace fpldpc_compat {
inline void check(int st, const char *what) {
    if (st != FPLDPC_OK) throw fpldpc_error(st, std::string(what) + ": " + fpldpc_last_error());
}
}  // namespace fpldpc_compat

// ArrayLDPCMacro.h:40 -- the FSM states (the same values).  decode_fixpoint follows the reference's
// state machine across calls (ArrayLDPC_Decoder.cpp:443-488, :621-630; see decode_fixpoint).
enum FPLDPC_FSMState { IDLE, PCV, V2C, SXOR, C2V, SIMEND };

class FP_Decoder {
   public:
    FP_Decoder() { fpldpc_params_default(&params_); }
    explicit FP_Decoder(const fpldpc_params &p) : params_(p) {}
    ~FP_Decoder() { release(); }
    FP_Decoder(const FP_Decoder &) = delete;
    FP_Decoder &operator=(const FP_Decoder &) = delete;

    // ReadH (ArrayLDPC_Decoder.cpp:642-674).
    void ReadH(const char *path = "H_802.11_IndZero.txt") {
        fpldpc_code_t c = nullptr;
        fpldpc_compat::check(fpldpc_code_load_alist(path, &c), "ReadH");
        setCode(c);
    }
    // Takes ownership of a code built by fpldpc_code_* (e.g. the native array / 802.11n codes).
    void setCode(fpldpc_code_t c) {
        release();
        code_ = c;
        int32_t d[8];
        fpldpc_compat::check(fpldpc_code_dims(code_, d), "code dims");
        n_ = d[0];
        m_ = d[1];
        edge_ram_.assign((size_t)d[3] * m_, 0);  // EdgeRAM[dc_max] x m (a zeroed static object's)
        post_.assign(n_, 0);
        postf_.assign(n_, 0.0);
        hard_.assign(n_, 0);
        true_cw_.assign(n_, 0);
    }
    fpldpc_code_t code() const { return code_; }
    int length() const { return n_; }

    // decode_general_fp (ArrayLDPC_Decoder.cpp:18-171): returns the iteration count.  Like the
    // reference it initialises the edge RAM from the LLRs and leaves its final messages there.
    int decode_general_fp(const int *LLR) { return decode_one(LLR, false, false); }
    // decode_fixpoint (:422-639): the same decode preceded by the channel-syndrome pre-check
    // (:443-450) -- 0 returned, hard decision = channel decision, posteriors and edge RAM of the
    // previous call kept.  The FSM, as the reference: the pre-check comes first and leaves the state
    // alone; in state PCV the edge RAM is initialised from the LLRs (:462-485); in state PCV or C2V
    // the iterations run (:488) and end in IDLE (syndrome met) or C2V (MAX_ITER reached, :621-630).
    // In C2V without setState(PCV) they continue from the edge RAM the previous decode left, with
    // this frame's LLRs in the variable-node phase (fpldpc_decode_frame, keep_edges = 1).  In IDLE
    // (or V2C / SXOR / SIMEND) the loop does not run: 0 with the channel decision and the previous
    // posteriors.
    int decode_fixpoint(const int *LLR) {
        if (state_ != PCV && state_ != C2V) {
            hardDecision(LLR);  // the pre-check's channel decision (:443)
            return 0;
        }
        uint8_t ok = 0;
        const int it = decode_one(LLR, true, state_ == C2V, &ok);
        if (it > 0) state_ = ok ? IDLE : C2V;  // (it == 0: the pre-check passed; the state stays)
        return it;
    }
    // Batch extension: B frames [B][n] (host), outputs optional (NULL).  Returns 0.
    int decode_batch(const int *LLR, int B, int *iters, uint8_t *hard_bits, int *post, bool fixpoint = false) {
        fpldpc_decoder_t d = dec(fixpoint);
        const int hw = (n_ + 31) / 32;
        std::vector<uint32_t> hard(hard_bits ? (size_t)B * hw : 0);
        fpldpc_compat::check(fpldpc_decode_host(d, LLR, FPLDPC_LLR_I32, B, hard_bits ? hard.data() : nullptr, iters,
                                                nullptr, post, nullptr, nullptr),
                             "decode_batch");
        if (hard_bits)
            for (int b = 0; b < B; b++)
                for (int v = 0; v < n_; v++) hard_bits[(size_t)b * n_ + v] = (hard[(size_t)b * hw + v / 32] >> (v % 32)) & 1;
        return 0;
    }

    // decode_general (:735-933): the floating-point BP decoder on unquantised double LLRs; returns
    // the iteration count, posteriors via getPost (fpldpc_decode_float: BER-level parity).
    int decode_general(const double *LLR) {
        fpldpc_decoder_t d = dec(false);
        const int hw = (n_ + 31) / 32;
        std::vector<uint32_t> hard(hw);
        int32_t it = 0;
        fpldpc_compat::check(fpldpc_decode_float_host(d, LLR, 1, hard.data(), &it, nullptr, postf_.data(), nullptr,
                                                      nullptr),
                             "decode_general");
        for (int v = 0; v < n_; v++) hard_[v] = (hard[v / 32] >> (v % 32)) & 1;
        return it;
    }
    // sxor(double, double) (:724-732), the exact Jacobian box-plus (host evaluation).
    static double sxor(double x, double y) {
        const double v1 = std::fabs(x), v2 = std::fabs(y);
        const double sum_abs = v1 + v2, diff_abs = std::fabs(v1 - v2);
        const int s = (x > 0 ? 1 : -1) * (y > 0 ? 1 : -1);
        return s * ((v2 < v1 ? v2 : v1) + std::log(1 + std::exp(-sum_abs)) - std::log(1 + std::exp(-diff_abs)));
    }
    double getPost(int addr) const { return postf_.at(addr); }  // ArrayLDPCMacro.h:149
    void wrtPost(int addr, double v) { postf_.at(addr) = v; }   // :153
    // checkPost (:335-372) on the double posteriors held: 0 pass, 1 fail.
    int checkPost() {
        std::vector<uint8_t> b(n_);
        for (int i = 0; i < n_; i++) hard_[i] = b[i] = postf_[i] > 0 ? 0 : 1;
        return syndrome(b.data());
    }

    int getPost_fp(int addr) const { return post_.at(addr); }  // ArrayLDPCMacro.h:138
    // EdgeRAM[k].BRAM_fp[c] (ArrayLDPCMacro.h:94, :162): the edge RAM between calls
    int getEdge_fp(int k, int c) const { return edge_ram_.at((size_t)k * m_ + c); }
    int getDecoded(int addr) const { return hard_.at(addr); }
    int getState() { return state_; }
    void setState(int s) { state_ = s; }
    void wrtPost(int addr, int v) { post_.at(addr) = v; }

    // setInfoBit (:178-197): LSB-first unpacking of the info char stream (k = info length).
    void setInfoBit(const char *in, int in_len, int k = -1) {
        if (k < 0) k = n_ - rank();
        true_info_.assign(k, 0);
        fpldpc_compat::check(fpldpc_unpack_info_bytes(in, in_len, k, true_info_.data()), "setInfoBit");
    }
    void setInfoIndex(const int *in, int k = -1) {  // :698-705
        if (k < 0) k = (int)true_info_.size();
        info_index_.assign(in, in + k);
    }
    void setCodeword(const int *in) { true_cw_.assign(in, in + n_); }  // :199-206
    // calculateBER (:707-722): ACCUMULATES into BitError until resetBER().
    int calculateBER() {
        for (size_t i = 0; i < info_index_.size(); i++)
            if (hard_.at(info_index_[i]) != (int)true_info_.at(i)) bit_error_++;
        return bit_error_;
    }
    void resetBER() { bit_error_ = 0; }
    // hardDecision (:270-294): DecodedCodeword = in > 0 ? 0 : 1, returns 1 if H fails.
    int hardDecision(const int *in) {
        std::vector<uint8_t> b(n_);
        for (int i = 0; i < n_; i++) hard_[i] = b[i] = in[i] > 0 ? 0 : 1;
        return syndrome(b.data());
    }
    // checkPost_fp_general (:296-333) on the posteriors held: 0 pass, 1 fail.
    int checkPost_fp_general() {
        std::vector<uint8_t> b(n_);
        for (int i = 0; i < n_; i++) hard_[i] = b[i] = post_[i] > 0 ? 0 : 1;
        return syndrome(b.data());
    }
    int check() { return syndrome_of(true_cw_); }  // :234-268 on TrueCodeword
    // check_fp (:210-232): 0 if the hard bits in[n] satisfy H, 1 if not.  The reference indexes
    // j + k*NUM_VGRP + shift without the mod-p wrap (out of range for most (j, shift)); this is the
    // syndrome it means, over the code's own check lists.
    int check_fp(const int *in) {
        std::vector<uint8_t> b(n_);
        for (int i = 0; i < n_; i++) b[i] = (uint8_t)(in[i] & 1);
        return syndrome(b.data());
    }
    // checkPost_fp (:375-420, array-code ROM addressing) == checkPost_fp_general on these codes
    int checkPost_fp() { return checkPost_fp_general(); }
    // ArrayLDPCMacro.h:218-243 helpers: sgn(0) = -1; fmin/fmax keep the reference's tie rule
    static int sgn(int x) { return x > 0 ? 1 : -1; }
    static int sgn(double x) { return x > 0 ? 1 : -1; }
    static int fmin(int x, int y) { return x <= y ? x : y; }
    static double fmin(double x, double y) { return x <= y ? x : y; }
    static int fmax(int x, int y) { return x >= y ? x : y; }
    // sxor (:677-694), the fixed-point box-plus, with this decoder's FRAC_WIDTH / WIDTH_MASK.
    int sxor(int x, int y) const {
        const int C = (int)((5.0 / 8.0) * (1 << params_.frac_bits));
        const int v1 = std::abs(x), v2 = std::abs(y);
        const int sum = (v1 + v2) & params_.width_mask, diff = std::abs(v1 - v2) & params_.width_mask;
        int p1 = C - (sum >> 2), p2 = C - (diff >> 2);
        p1 = p1 > 0 ? p1 : 0;
        p2 = p2 > 0 ? p2 : 0;
        const int s = (x > 0 ? 1 : -1) * (y > 0 ? 1 : -1);  // sgn, ArrayLDPCMacro.h:222-224
        return s * ((v1 < v2 ? v1 : v2) + p1 - p2);
    }
    double getRate() const {  // ROM::getRate for array codes (ArrayLDPCMacro.h:60)
        double r = 0;
        fpldpc_compat::check(fpldpc_code_rate(code_, &r), "getRate");
        return r;
    }
    int rank() const {
        int32_t d[8];
        fpldpc_compat::check(fpldpc_code_dims(code_, d), "code dims");
        return d[6];
    }
    fpldpc_decoder_t device_decoder(bool fixpoint) { return dec(fixpoint); }
    const fpldpc_params &params() const { return params_; }

   private:
    // One frame through the stateful path: the edge RAM (FP_Decoder::EdgeRAM, ArrayLDPCMacro.h:162)
    // is this object's, shared by decode_general_fp and decode_fixpoint as in the reference.
    int decode_one(const int *LLR, bool fixpoint, bool keep_edges, uint8_t *syn_ok = nullptr) {
        fpldpc_decoder_t d = dec(fixpoint);
        const int hw = (n_ + 31) / 32;
        std::vector<uint32_t> hard(hw);
        int32_t it = 0;
        // post_ and edge_ram_ seed the device copies, so a pre-check pass leaves them untouched (:443-450)
        fpldpc_compat::check(fpldpc_decode_frame_host(d, LLR, keep_edges ? 1 : 0, edge_ram_.data(), hard.data(), &it,
                                                      syn_ok, post_.data()),
                             fixpoint ? "decode_fixpoint" : "decode_general_fp");
        for (int v = 0; v < n_; v++) hard_[v] = (hard[v / 32] >> (v % 32)) & 1;
        return it;
    }
    fpldpc_decoder_t dec(bool fixpoint) {
        if (!code_) throw fpldpc_error(FPLDPC_ERR_ARG, "FP_Decoder: no code (call ReadH or setCode)");
        fpldpc_decoder_t &d = fixpoint ? dec_fix_ : dec_gen_;
        if (!d) {
            fpldpc_params p = params_;
            p.precheck = fixpoint ? 1 : 0;
            fpldpc_compat::check(fpldpc_decoder_create(code_, &p, &d), "decoder_create");
        }
        return d;
    }
    int syndrome(const uint8_t *bits) {
        const int r = fpldpc_code_syndrome_host(code_, bits);
        fpldpc_compat::check(r < 0 ? r : 0, "syndrome");
        return r;
    }
    int syndrome_of(const std::vector<int> &v) {
        std::vector<uint8_t> b(v.begin(), v.end());
        return syndrome(b.data());
    }
    void release() {
        if (dec_gen_) fpldpc_decoder_destroy(dec_gen_);
        if (dec_fix_) fpldpc_decoder_destroy(dec_fix_);
        if (code_) fpldpc_code_free(code_);
        dec_gen_ = dec_fix_ = nullptr;
        code_ = nullptr;
    }

    fpldpc_params params_{};
    fpldpc_code_t code_ = nullptr;
    fpldpc_decoder_t dec_gen_ = nullptr, dec_fix_ = nullptr;
    int n_ = 0, m_ = 0, state_ = IDLE, bit_error_ = 0;
    std::vector<int> post_, hard_, true_cw_;
    std::vector<int32_t> edge_ram_;  // edge_ram_[k * m + c]: v2c on slot k of check c (fpldpc_decode_frame)
    std::vector<double> postf_;
    std::vector<uint8_t> true_info_;
    std::vector<int> info_index_;
};

class FP_Encoder {
   public:
    // FP_Encoder(char *Filename, int flag) (ArrayLDPC_Encoder.cpp:34-157): the reference's G file.
    FP_Encoder(const char *g_file, int /*verbose*/) { fpldpc_compat::check(fpldpc_encoder_load_g(g_file, &e_), "FP_Encoder"); init(); }
    // Native: systematic encoder derived from H (same positions / codewords as the G files).
    explicit FP_Encoder(fpldpc_code_t code) { fpldpc_compat::check(fpldpc_encoder_from_code(code, &e_), "FP_Encoder"); init(); }
    ~FP_Encoder() { fpldpc_encoder_free(e_); }
    FP_Encoder(const FP_Encoder &) = delete;
    FP_Encoder &operator=(const FP_Encoder &) = delete;
    // encode(char *in, int in_len) (:160-225): returns the codeword length.
    int encode(const char *in, int in_len) {
        std::vector<uint8_t> info(k_);
        fpldpc_compat::check(fpldpc_unpack_info_bytes(in, in_len, k_, info.data()), "encode");
        std::vector<uint8_t> cw(n_);
        fpldpc_compat::check(fpldpc_encoder_encode_host(e_, info.data(), 1, cw.data(), 1), "encode");
        codeword_.assign(cw.begin(), cw.end());
        return n_;
    }
    // encode(char *in, char *out, int in_len) (:228-320): also packs the codeword LSB-first into
    // out, XORed into the caller's (zeroed) bytes as the reference does; returns ceil(n / 8), the
    // bytes written (the reference's return value is derived from the WiFi enum and its console
    // dump of every byte is not reproduced).
    int encode(const char *in, char *out, int in_len) {
        encode(in, in_len);
        for (int v = 0; v < n_; v++) out[v / 8] = (char)(out[v / 8] ^ (codeword_[v] << (v % 8)));
        return (n_ + 7) / 8;
    }
    int getCodeword(int addr) const { return codeword_.at(addr); }
    int getInfoIndex(int addr) const { return info_index_.at(addr); }
    int length() const { return n_; }
    int info_length() const { return k_; }
    fpldpc_encoder_t handle() const { return e_; }

   private:
    void init() {
        int32_t d[3];
        fpldpc_compat::check(fpldpc_encoder_dims(e_, d), "encoder dims");
        n_ = d[0];
        k_ = d[1];
        info_index_.resize(k_);
        fpldpc_compat::check(fpldpc_encoder_info_index(e_, info_index_.data(), nullptr), "encoder info index");
        codeword_.assign(n_, 0);
    }
    fpldpc_encoder_t e_ = nullptr;
    int n_ = 0, k_ = 0;
    std::vector<int> info_index_, codeword_;
};

// PerfTest.h:4-11, re-implemented over the batched GPU decoder (fpldpc_perftest.cpp).  They print
// the reference's console lines.  Data files are looked up in the working directory exactly as the
// reference does ("H_802.11_IndZero.txt", "H_802.11_IndZerog.txt", "G_array_forward.txt"); when a
// file is absent the built-in code construction / native encoder is used instead.
void noMoreMemory();
int ArrayLDPC_Debug();                                   // PerfTest.cpp:217-316 (4.5 dB, array code)
int ArrayLDPC_Debug_Wifi();                              // :23-140, reads Eb/N0 from stdin like the reference
int ArrayLDPC_Debug_Wifi(double EbN0_dB);                // non-interactive
int ArrayLDPC_PerfTest(double db_start, double db_end, double db_step, char *Filename);  // :433-517
int ArrayLDPC_TimeTrial(double db, int MaxPckNum, char *Filename);                      // :520-607
int DecodeTrial(double EbN0_dB, int MaxPacket);          // :148-192
int EncodeTrial(char *info, int MaxPacket);              // :193-215
int ArrayLDPC_Debug_Shorten(int short_len);              // :318-431
