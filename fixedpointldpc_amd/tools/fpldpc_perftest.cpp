// fpldpc_perftest -- command-line driver of the PerfTest.h functions (fpldpc_compat.hpp), the
// counterpart of the reference's Wrapper.cpp main (Wrapper.cpp:17-101), non-interactive.
//   fpldpc_perftest wifi [EbN0]          ArrayLDPC_Debug_Wifi   (stdin prompt when EbN0 is omitted)
//   fpldpc_perftest array                ArrayLDPC_Debug        (4.5 dB, decode_fixpoint)
//   fpldpc_perftest shorten LEN          ArrayLDPC_Debug_Shorten
//   fpldpc_perftest decode_trial EbN0 N  DecodeTrial
//   fpldpc_perftest encode_trial N       EncodeTrial
//   fpldpc_perftest perftest db0 db1 step FILE   ArrayLDPC_PerfTest
//   fpldpc_perftest timetrial db N FILE          ArrayLDPC_TimeTrial
//   fpldpc_perftest wifi_float db N              WiFi loop through decode_general (floating point)
//   fpldpc_perftest frames ALIST LLR OUT FIX MAX_ITER MASK RESET [FILL]
//                                                the reference's per-frame FP_Decoder call sequence
//                                                over a file of LLR vectors (see frames() below)
//   fpldpc_perftest frame_time ALIST LLR FIX MAX_ITER MASK [WARM]
//                                                per-call latency of that sequence (frame_time())
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <fstream>
#include <vector>

#include "fpldpc_compat.hpp"

// wifi_float EbN0 nframes: the WiFi harness loop (PerfTest.cpp:97-135) driven through the
// floating-point decoder FP_Decoder::decode_general (ArrayLDPC_Decoder.cpp:735-933) one frame at
// a time, unquantised LLRs; prints the per-frame iteration counts and the harness result line.
static int wifi_float(double EbN0_dB, int frames) {
    static const char kInfo[122] = "OMG  how long   dd   should this string be to make it 243";  // PerfTest.cpp:33
    FP_Decoder Decoder;
    fpldpc_code_t c = nullptr;
    fpldpc_compat::check(fpldpc_code_wifi_1944_r12(&c), "code");
    Decoder.setCode(c);
    fpldpc_encoder_t e = nullptr;
    fpldpc_compat::check(fpldpc_encoder_from_code(c, &e), "encoder");
    int32_t dims[3];
    fpldpc_compat::check(fpldpc_encoder_dims(e, dims), "encoder");
    const int n = dims[0], k = dims[1];
    std::vector<uint8_t> bits(k), cw(n);
    std::vector<int32_t> idx(k);
    fpldpc_compat::check(fpldpc_unpack_info_bytes(kInfo, 122, k, bits.data()), "setInfoBit");
    fpldpc_compat::check(fpldpc_encoder_encode_host(e, bits.data(), 1, cw.data(), 1), "encode");
    fpldpc_compat::check(fpldpc_encoder_info_index(e, idx.data(), nullptr), "info index");
    fpldpc_encoder_free(e);
    Decoder.setInfoBit(kInfo, 122, k);
    Decoder.setInfoIndex(idx.data(), k);
    const double snr = 2 * pow(10.0, EbN0_dB / 10) * 0.5, sigma = std::sqrt(1 / snr);
    std::vector<double> llr(n);
    double biterror = 0, pckerror = 0;
    for (int f = 0; f < frames; f++) {
        fpldpc_compat::check(fpldpc_channel_llr_host(123456789, f, 1, n, snr, sigma, 4, cw.data(), llr.data(),
                                                     FPLDPC_LLR_F64, 1),
                             "channel");
        const int it = Decoder.decode_general(llr.data());
        Decoder.resetBER();
        const int blk = Decoder.calculateBER();
        if (blk > 0) pckerror++;
        biterror += blk;
        std::cout << it << ", ";
    }
    std::cout << "\n" << biterror << " " << pckerror << " " << frames << std::endl;
    std::cout << "post0 " << Decoder.getPost(0) << " " << Decoder.getPost(1) << std::endl;
    return 0;
}

// frames: the reference's per-frame call sequence (PerfTest.cpp:121-130 for the WiFi loop, :505-507
// for ArrayLDPC_PerfTest) through FP_Decoder, one GPU decode per call:
//   ReadH(alist), setInfoBit(a stream of FILL bytes, default 0), setInfoIndex(the native
//   encoder's info positions), then
//   per frame setState(PCV); decode_general_fp or decode_fixpoint (fix = 1); resetBER() when
//   f % reset == 0 (else calculateBER keeps accumulating, ArrayLDPCMacro.h:146); calculateBER();
//   getPost_fp(0..n-1); getDecoded(0..n-1).
// llr_file: int32 [frames][n] (frames = file size / 4n).  out_file (int32): k, info_index[k], then
// per frame: return value, calculateBER(), posteriors[n], hard decisions[n].
static int frames(const char *alist, const char *llr_file, const char *out_file, int fix, int max_iter, int mask,
                  int reset, int fill) {
    fpldpc_params p;
    fpldpc_params_default(&p);
    p.max_iter = max_iter;
    p.width_mask = mask;
    FP_Decoder Decoder(p);
    Decoder.ReadH(alist);
    const int n = Decoder.length();
    FP_Encoder Encoder(Decoder.code());
    const int k = Encoder.info_length();
    std::vector<char> stream((k + 7) / 8, (char)fill);
    Decoder.setInfoBit(stream.data(), (int)stream.size());
    std::vector<int> idx(k);
    for (int i = 0; i < k; i++) idx[i] = Encoder.getInfoIndex(i);
    Decoder.setInfoIndex(idx.data());
    std::vector<int32_t> all;
    {
        std::ifstream f(llr_file, std::ios::binary | std::ios::ate);
        const size_t bytes = (size_t)f.tellg();
        all.resize(bytes / 4);
        f.seekg(0);
        f.read((char *)all.data(), (std::streamsize)(all.size() * 4));
        if (!f || all.size() % n) throw fpldpc_error(FPLDPC_ERR_ARG, "frames: LLR file size is not a multiple of 4n");
    }
    std::ofstream out(out_file, std::ios::binary);
    auto put = [&](int32_t v) { out.write((const char *)&v, 4); };
    put(k);
    for (int i = 0; i < k; i++) put(idx[i]);
    const int nf = (int)(all.size() / n);
    for (int f = 0; f < nf; f++) {
        Decoder.setState(PCV);
        const int *L = &all[(size_t)f * n];
        const int it = fix ? Decoder.decode_fixpoint(L) : Decoder.decode_general_fp(L);
        if (reset > 0 && f % reset == 0) Decoder.resetBER();
        put(it);
        put(Decoder.calculateBER());
        for (int v = 0; v < n; v++) put(Decoder.getPost_fp(v));
        for (int v = 0; v < n; v++) put(Decoder.getDecoded(v));
    }
    if (!out) throw fpldpc_error(FPLDPC_ERR_ARG, "frames: cannot write the output file");
    std::cout << nf << " frames" << std::endl;
    return 0;
}

// fsm: decode_fixpoint over a file of LLR vectors with setState(PCV) before frame f only when
// flags[f] == '1' -- the reference's FSM across calls (ArrayLDPC_Decoder.cpp:443-488, :621-630).
// In state C2V without PCV a call continues from the edge RAM the previous decode left (:462-488).
// out_file (int32) per frame: return value, getState(), posteriors[n], hard decisions[n], and the
// edge RAM the call left, getEdge_fp(k, c) for k < dc_max, c < m (EdgeRAM[k].BRAM_fp[c]).
static int fsm(const char *alist, const char *llr_file, const char *out_file, int max_iter, int mask, const char *flags) {
    fpldpc_params p;
    fpldpc_params_default(&p);
    p.max_iter = max_iter;
    p.width_mask = mask;
    FP_Decoder Decoder(p);
    Decoder.ReadH(alist);
    const int n = Decoder.length();
    int32_t dims[8];
    fpldpc_compat::check(fpldpc_code_dims(Decoder.code(), dims), "code dims");
    const int m = dims[1], dc = dims[3];
    std::vector<int32_t> all;
    {
        std::ifstream f(llr_file, std::ios::binary | std::ios::ate);
        all.resize((size_t)f.tellg() / 4);
        f.seekg(0);
        f.read((char *)all.data(), (std::streamsize)(all.size() * 4));
        if (!f || all.size() % n || all.size() / n != strlen(flags))
            throw fpldpc_error(FPLDPC_ERR_ARG, "fsm: LLR file size is not 4n per flag");
    }
    std::ofstream out(out_file, std::ios::binary);
    auto put = [&](int32_t v) { out.write((const char *)&v, 4); };
    const int nf = (int)strlen(flags);
    for (int f = 0; f < nf; f++) {
        if (flags[f] == '1') Decoder.setState(PCV);
        const int it = Decoder.decode_fixpoint(&all[(size_t)f * n]);
        put(it);
        put(Decoder.getState());
        for (int v = 0; v < n; v++) put(Decoder.getPost_fp(v));
        for (int v = 0; v < n; v++) put(Decoder.getDecoded(v));
        for (int k = 0; k < dc; k++)
            for (int c = 0; c < m; c++) put(Decoder.getEdge_fp(k, c));
    }
    return out ? 0 : 1;
}

// frame_time: the per-frame drop-in call's latency -- the reference's callers decode one frame per
// call (PerfTest.cpp:121-128, :178-182, :304).  Over a file of int32 LLR vectors: setState(PCV) and
// decode_general_fp (fix = 0) or decode_fixpoint (fix = 1) per frame, each call timed on the host
// clock (the whole call: staging, the flood_edges launch, the copies back, the synchronisation), after
// WARM untimed calls.  Prints one JSON line: per-call microseconds (mean / median / min / max), the
// iteration sum.
static int frame_time(const char *alist, const char *llr_file, int fix, int max_iter, int mask, int warm) {
    fpldpc_params p;
    fpldpc_params_default(&p);
    p.max_iter = max_iter;
    p.width_mask = mask;
    FP_Decoder Decoder(p);
    Decoder.ReadH(alist);
    const int n = Decoder.length();
    std::vector<int32_t> all;
    {
        std::ifstream f(llr_file, std::ios::binary | std::ios::ate);
        all.resize((size_t)f.tellg() / 4);
        f.seekg(0);
        f.read((char *)all.data(), (std::streamsize)(all.size() * 4));
        if (!f || all.size() % n) throw fpldpc_error(FPLDPC_ERR_ARG, "frame_time: LLR file size is not a multiple of 4n");
    }
    const int nf = (int)(all.size() / n);
    auto call = [&](int f) {
        Decoder.setState(PCV);
        const int *L = &all[(size_t)f * n];
        return fix ? Decoder.decode_fixpoint(L) : Decoder.decode_general_fp(L);
    };
    for (int w = 0; w < warm; w++) call(w % nf);
    std::vector<double> us(nf);
    long long iters = 0;
    for (int f = 0; f < nf; f++) {
        const auto t0 = std::chrono::steady_clock::now();
        iters += call(f);
        us[f] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    std::vector<double> s = us;
    std::sort(s.begin(), s.end());
    double sum = 0;
    for (double x : us) sum += x;
    printf("{\"frames\": %d, \"iterations\": %lld, \"us_mean\": %.2f, \"us_median\": %.2f, \"us_min\": %.2f, "
           "\"us_max\": %.2f, \"us_total\": %.1f}\n",
           nf, iters, sum / nf, s[nf / 2], s[0], s[nf - 1], sum);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::cerr << "usage: fpldpc_perftest {wifi|array|shorten|decode_trial|encode_trial|perftest|timetrial|wifi_float} ...\n";
        return 2;
    }
    const std::string m = argv[1];
    try {
        if (m == "wifi") return argc > 2 ? ArrayLDPC_Debug_Wifi(atof(argv[2])) : ArrayLDPC_Debug_Wifi();
        if (m == "array") return ArrayLDPC_Debug();
        if (m == "shorten" && argc > 2) return ArrayLDPC_Debug_Shorten(atoi(argv[2]));
        if (m == "decode_trial" && argc > 3) return DecodeTrial(atof(argv[2]), atoi(argv[3]));
        if (m == "encode_trial" && argc > 2) {
            char info[248] = "OMG how long should this string be to make it 248";
            return EncodeTrial(info, atoi(argv[2]));
        }
        if (m == "perftest" && argc > 5) return ArrayLDPC_PerfTest(atof(argv[2]), atof(argv[3]), atof(argv[4]), argv[5]);
        if (m == "wifi_float" && argc > 3) return wifi_float(atof(argv[2]), atoi(argv[3]));
        if (m == "frames" && argc > 8)
            return frames(argv[2], argv[3], argv[4], atoi(argv[5]), atoi(argv[6]), (int)strtol(argv[7], nullptr, 0),
                          atoi(argv[8]), argc > 9 ? (int)strtol(argv[9], nullptr, 0) : 0);
        if (m == "fsm" && argc > 7)
            return fsm(argv[2], argv[3], argv[4], atoi(argv[5]), (int)strtol(argv[6], nullptr, 0), argv[7]);
        if (m == "frame_time" && argc > 6)
            return frame_time(argv[2], argv[3], atoi(argv[4]), atoi(argv[5]), (int)strtol(argv[6], nullptr, 0),
                              argc > 7 ? atoi(argv[7]) : 20);
        if (m == "timetrial" && argc > 4) return ArrayLDPC_TimeTrial(atof(argv[2]), atoi(argv[3]), argv[4]);
    } catch (const fpldpc_error &e) {
        std::cerr << "fpldpc_perftest: " << e.what() << "\n";
        return 1;
    }
    std::cerr << "fpldpc_perftest: bad arguments\n";
    return 2;
}
