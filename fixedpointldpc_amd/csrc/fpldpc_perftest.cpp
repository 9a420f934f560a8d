// fpldpc_perftest.cpp -- PerfTest.h (PerfTest.cpp) re-implemented over the batched GPU decoder.
//
// Each function keeps the reference's inputs, channel, stop rule and console output; the frame loop
// is fpldpc_ber_sim (ordered accounting, so "stop at the 100th frame error" lands on the same frame).
// Non-interactive overloads take what the reference reads from cin.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <vector>

#include "fpldpc_compat.hpp"

namespace {

// Info streams of the harness (test vectors): PerfTest.cpp:33 (WiFi, char[122]) and :221-224
// (array code, char[248]; the literal's line continuations keep the tabs of the next line).
const char kWifiInfo[122] = "OMG  how long   dd   should this string be to make it 243";
const char kArrayInfo[248] =
    "OMG how long should this string be to make it 248, just imagine that. \t\t\t\t\t\t\t\t   I guess it's still "
    "not long enough. Let's see. This is a testing string \t\t\t\t\t\t\t\t\tfor a lot of characters so that we have "
    "some random bit stream that's\t\t\t\t\t\t\t\t\tcorrect";

bool exists(const char *p) {
    std::ifstream f(p);
    return (bool)f;
}

fpldpc_code_t wifi_code() {
    fpldpc_code_t c = nullptr;
    if (exists("H_802.11_IndZero.txt"))
        fpldpc_compat::check(fpldpc_code_load_alist("H_802.11_IndZero.txt", &c), "ReadH");
    else
        fpldpc_compat::check(fpldpc_code_wifi_1944_r12(&c), "wifi code");
    return c;
}

fpldpc_code_t array_code() {
    fpldpc_code_t c = nullptr;
    if (exists("H_array_p47_r5_forward.txt"))
        fpldpc_compat::check(fpldpc_code_load_alist("H_array_p47_r5_forward.txt", &c), "ReadH");
    else
        fpldpc_compat::check(fpldpc_code_array(47, 5, 1, &c), "array code");
    return c;
}

std::unique_ptr<FP_Encoder> encoder_for(const char *g_file, fpldpc_code_t code) {
    if (exists(g_file)) return std::unique_ptr<FP_Encoder>(new FP_Encoder(g_file, 0));
    return std::unique_ptr<FP_Encoder>(new FP_Encoder(code));
}

// Devices the harness loop shards over, opt-in so that the reference's console lines
// keep their single-decoder meaning by default: FPLDPC_SIM_DEVICES unset = one decoder on the
// current device (the FP_Decoder's own); "all" = every visible device; a list of ordinals
// ("0,1,2,3"; repeating one, "0,0,0", runs several decoders on one device -- the multi-rank path
// rehearsed on a 1-GPU box).  An empty result means the default.
std::vector<int> sim_devices() {
    std::vector<int> devs;
    const char *e = std::getenv("FPLDPC_SIM_DEVICES");
    if (!e || !*e) return devs;
    if (!strcmp(e, "all")) {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count < 1) count = 1;
        for (int d = 0; d < count; d++) devs.push_back(d);
        return devs;
    }
    for (const char *p = e; *p;) {
        char *end = nullptr;
        const long d = std::strtol(p, &end, 10);
        if (end == p) break;
        devs.push_back((int)d);
        p = *end ? end + 1 : end;
    }
    return devs;
}

// One decoder per listed device (rank r on devs[r], rank 0 included), same code / params.
struct RankDecoders {
    std::vector<fpldpc_decoder_t> d;
    RankDecoders(FP_Decoder &dec, bool fixpoint, const std::vector<int> &devs) {
        for (size_t i = 0; i < devs.size(); i++) {
            fpldpc_params p = dec.params();
            p.precheck = fixpoint ? 1 : 0;
            p.device = devs[i];
            fpldpc_decoder_t x = nullptr;
            const int st = fpldpc_decoder_create(dec.code(), &p, &x);
            if (st != FPLDPC_OK) {
                const std::string msg = std::string("decoder_create: ") + fpldpc_last_error();
                for (auto y : d) fpldpc_decoder_destroy(y);
                throw fpldpc_error(st, msg);
            }
            d.push_back(x);
        }
    }
    ~RankDecoders() {
        for (auto x : d) fpldpc_decoder_destroy(x);
    }
};

// One BER run of the harness loop.  cw: transmitted codeword (NULL = all-zero).
fpldpc_sim_result run(FP_Decoder &dec, bool fixpoint, double snr, const std::vector<uint8_t> *cw,
                      const std::vector<int32_t> *info_idx, const std::vector<uint8_t> *info_bits, int64_t max_fe,
                      int64_t max_frames, int count_mode, const std::vector<int32_t> *forced = nullptr,
                      int forced_llr = 0, void (*on_frame)(void *, int64_t, int32_t, int64_t) = nullptr) {
    fpldpc_sim_params sp;
    fpldpc_sim_params_default(&sp);
    sp.snr = snr;
    sp.sigma = std::sqrt(1 / snr);
    sp.frac_bits = dec.params().frac_bits;
    sp.codeword = cw ? cw->data() : nullptr;
    if (info_idx) {
        sp.info_index = info_idx->data();
        sp.info_bits = info_bits->data();
        sp.k = (int32_t)info_idx->size();
    }
    if (forced) {
        sp.forced_index = forced->data();
        sp.n_forced = (int32_t)forced->size();
        sp.forced_llr = forced_llr;
    }
    sp.max_frame_errors = max_fe;
    sp.max_frames = max_frames;
    sp.count_mode = count_mode;
    sp.on_frame = on_frame;
    // LLRs generated on the device (bit-exact with the host channel over the whole KAT-W stream,
    // tests/test_gpu_gen.py); FPLDPC_HOST_CHANNEL=1 generates them on host threads instead
    const char *hc = std::getenv("FPLDPC_HOST_CHANNEL");
    sp.device_channel = !(hc && *hc && *hc != '0');
    fpldpc_sim_result r{};
    const std::vector<int> devs = sim_devices();
    if (devs.empty()) {
        fpldpc_compat::check(fpldpc_ber_sim(dec.device_decoder(fixpoint), &sp, &r), "ber_sim");
        return r;
    }
    RankDecoders rd(dec, fixpoint, devs);
    int32_t used = 0;
    fpldpc_compat::check(fpldpc_ber_sim_multi(rd.d.data(), (int32_t)rd.d.size(), &sp, FPLDPC_COLL_AUTO, &r, &used),
                         "ber_sim_multi");
    std::cerr << "frame loop sharded over " << rd.d.size() << " decoders (" << (used == FPLDPC_COLL_RCCL ? "RCCL" : "host")
              << " exchange)" << std::endl;
    return r;
}

void print_result(double biterror, double pckerror, long Counter, int n) {
    // PerfTest.cpp:136-137 (BER divides by CWD_LENGTH)
    std::cout << biterror << " " << pckerror << " " << Counter << std::endl
              << " FER: " << pckerror / Counter << " BER: " << biterror / Counter / n << std::endl;
}

void print_iters(void *, int64_t, int32_t it, int64_t) { std::cout << it << ", "; }

bool touch(const char *Filename) {
    // ArrayLDPC_PerfTest / TimeTrial create <file> and <file>_log.txt, both left empty (:461-480)
    std::ofstream a(Filename);
    if (!a) {
        std::cerr << "failed to open " << Filename << std::endl;
        return false;
    }
    std::ofstream b(std::string(Filename) + "_log.txt");
    if (!b) {
        std::cerr << "failed to open " << Filename << "_log.txt" << std::endl;
        return false;
    }
    return true;
}

}  // namespace

void noMoreMemory() {
    std::cerr << "Unable to satisfy request for memory\n";
    abort();
}

int ArrayLDPC_Debug_Wifi(double EbN0_dB) {
    FP_Decoder Decoder;
    Decoder.setCode(wifi_code());
    auto Encoder = encoder_for("H_802.11_IndZerog.txt", Decoder.code());
    const double snr = 2 * pow(10.0, EbN0_dB / 10) * 0.5;  // PerfTest.cpp:62, rate hard-coded
    std::cout << "SNR is " << 10 * log10(snr) << " dB" << std::endl;
    const int k = Encoder->info_length();
    Decoder.setInfoBit(kWifiInfo, 122, k);
    std::vector<int32_t> idx(k);
    for (int i = 0; i < k; i++) idx[i] = Encoder->getInfoIndex(i);
    Encoder->encode(kWifiInfo, 122);
    std::vector<uint8_t> cw(Encoder->length()), bits(k);
    for (int i = 0; i < Encoder->length(); i++) cw[i] = (uint8_t)Encoder->getCodeword(i);
    fpldpc_compat::check(fpldpc_unpack_info_bytes(kWifiInfo, 122, k, bits.data()), "setInfoBit");
    const auto r = run(Decoder, false, snr, &cw, &idx, &bits, 100, 0, FPLDPC_COUNT_BITS);
    print_result((double)r.bit_errors, (double)r.frame_errors, (long)r.frames, Decoder.length());
    return 0;
}

int ArrayLDPC_Debug_Wifi() {
    double EbN0_dB = 3;
    std::cout << "EbNo in dB? ";
    std::cin >> EbN0_dB;
    return ArrayLDPC_Debug_Wifi(EbN0_dB);
}

static int array_debug(int short_len) {
    FP_Decoder Decoder;
    Decoder.setCode(array_code());
    auto Encoder = encoder_for("G_array_forward.txt", Decoder.code());
    const double EbN0_dB = 4.5;
    char info[248];
    memcpy(info, kArrayInfo, sizeof info);
    for (int i = 0; i < short_len && i < 248; i++) info[i] = 0;  // :360-366
    // :251-253; the shortened variant hard-codes the rate (1978 - 976) / 2209 (:354)
    const double snr = short_len > 0 ? 2 * pow(10.0, EbN0_dB / 10) * (1978.0 - 976.0) / 2209.0
                                     : 2 * pow(10.0, EbN0_dB / 10) * Decoder.getRate();
    std::cout << "SNR is " << 10 * log10(snr) << " dB" << std::endl;
    const int k = Encoder->info_length();
    std::vector<int32_t> idx(k);
    for (int i = 0; i < k; i++) idx[i] = Encoder->getInfoIndex(i);
    std::vector<uint8_t> bits(k);
    fpldpc_compat::check(fpldpc_unpack_info_bytes(info, 248, k, bits.data()), "setInfoBit");
    Encoder->encode(info, 248);
    std::vector<uint8_t> cw(Encoder->length());
    for (int i = 0; i < Encoder->length(); i++) cw[i] = (uint8_t)Encoder->getCodeword(i);
    std::vector<int32_t> forced(idx.begin(), idx.begin() + std::min(short_len, k));  // :410-414
    const auto r = run(Decoder, true, snr, &cw, &idx, &bits, 100, 0, FPLDPC_COUNT_BITS,
                       short_len > 0 ? &forced : nullptr, 7 * (1 << Decoder.params().frac_bits),
                       short_len > 0 ? print_iters : nullptr);
    print_result((double)r.bit_errors, (double)r.frame_errors, (long)r.frames, Decoder.length());
    return 0;
}

int ArrayLDPC_Debug() { return array_debug(0); }

int ArrayLDPC_Debug_Shorten(int short_len) { return array_debug(short_len); }

static int perf_or_time(double db, int64_t max_frames, char *Filename) {
    if (!touch(Filename)) exit(0);
    FP_Decoder Decoder;
    Decoder.setCode(array_code());
    const double snr = 2 * pow(10.0, db / 10) * Decoder.getRate();  // "EbN0" in :489-491
    // all-zero codeword; blkerror = decode_fixpoint's return value (:507-510, 596-600)
    const auto r = run(Decoder, true, snr, nullptr, nullptr, nullptr, max_frames > 0 ? 0 : 100, max_frames,
                       FPLDPC_COUNT_ITERS);
    print_result((double)r.bit_errors, (double)r.frame_errors, (long)r.frames, Decoder.length());
    return 0;
}

int ArrayLDPC_PerfTest(double db_start, double /*db_end*/, double /*db_step*/, char *Filename) {
    return perf_or_time(db_start, 0, Filename);  // the reference only ever runs db_start (:487)
}

int ArrayLDPC_TimeTrial(double db, int MaxPckNum, char *Filename) { return perf_or_time(db, MaxPckNum, Filename); }

int DecodeTrial(double EbN0_dB, int MaxPacket) {
    // :148-192: 100 all-zero-codeword frames, MaxPacket decode_fixpoint calls cycling over them --
    // here split over the devices of sim_devices() (packet p still decodes vector p % 100: every
    // rank's share but the last is a multiple of 100), one host thread per device, wall time from a
    // common start to the last rank's finish.
    FP_Decoder Decoder;
    Decoder.setCode(array_code());
    const int n = Decoder.length();
    const double snr = 2 * pow(10.0, EbN0_dB / 10) * Decoder.getRate();
    std::cout << "equivalent SNR is: " << 10 * log10(snr) << std::endl;
    std::vector<int32_t> llr100((size_t)100 * n);
    fpldpc_compat::check(fpldpc_channel_llr_host(123456789, 0, 100, n, snr, std::sqrt(1 / snr),
                                                 Decoder.params().frac_bits, nullptr, llr100.data(), FPLDPC_LLR_I32, 0),
                         "channel");
    std::vector<int> devs = sim_devices();
    if (devs.empty()) devs.push_back(-1);  // default: the FP_Decoder's own decoder, current device
    if (MaxPacket < 100 * (int)devs.size()) devs.resize(1);  // too few packets to split by whole tiles
    const int R = (int)devs.size();
    std::vector<int> share(R, 0);
    {
        const int per = (MaxPacket / 100 + R - 1) / R * 100;  // multiple of 100
        int left = MaxPacket;
        for (int r = 0; r < R; r++) {
            share[r] = std::min(per, left);
            left -= share[r];
        }
        share[R - 1] += left;
    }
    // device batch = the 100 vectors tiled (frame i uses vector i % 100); B is a multiple of 100, so
    // every launch starts at vector 0 like frame i = launch * B
    const int B = std::max(1, std::min(std::max(share[0], 1), 100 * 82));  // up to 8200 frames per launch
    std::vector<int32_t> tiled((size_t)B * n);
    for (int i = 0; i < B; i++) memcpy(&tiled[(size_t)i * n], &llr100[(size_t)(i % 100) * n], sizeof(int32_t) * n);
    std::unique_ptr<RankDecoders> own;
    std::vector<fpldpc_decoder_t> decs;
    if (devs[0] < 0) {
        decs.push_back(Decoder.device_decoder(true));
    } else {
        own.reset(new RankDecoders(Decoder, true, devs));
        decs = own->d;
    }
    std::vector<std::vector<int32_t>> its(R);
    std::vector<std::string> errs(R);
    std::mutex m;
    std::condition_variable cv;
    int ready = 0;
    std::chrono::steady_clock::time_point t0;
    auto rank = [&](int r) {
        void *d_llr = nullptr, *d_it = nullptr;
        try {
            if (devs[r] >= 0 && hipSetDevice(devs[r]) != hipSuccess) throw fpldpc_error(FPLDPC_ERR_HIP, "hipSetDevice");
            if (hipMalloc(&d_llr, tiled.size() * 4) != hipSuccess || hipMalloc(&d_it, (size_t)B * 4) != hipSuccess)
                throw fpldpc_error(FPLDPC_ERR_HIP, "DecodeTrial: hipMalloc");
            (void)hipMemcpy(d_llr, tiled.data(), tiled.size() * 4, hipMemcpyHostToDevice);
            {  // common start
                std::unique_lock<std::mutex> l(m);
                if (++ready == R) {
                    t0 = std::chrono::steady_clock::now();
                    cv.notify_all();
                } else {
                    cv.wait(l, [&] { return ready == R; });
                }
            }
            for (int done = 0; done < share[r]; done += B)
                fpldpc_compat::check(fpldpc_decode(decs[r], d_llr, FPLDPC_LLR_I32, std::min(B, share[r] - done), nullptr,
                                                   (int32_t *)d_it, nullptr, nullptr, nullptr, nullptr, nullptr),
                                     "DecodeTrial");
            if (hipDeviceSynchronize() != hipSuccess) throw fpldpc_error(FPLDPC_ERR_HIP, "DecodeTrial: synchronize");
            const int last = share[r] > 0 ? share[r] - (share[r] - 1) / B * B : 0;
            its[r].resize((size_t)last);
            if (last > 0 && hipMemcpy(its[r].data(), d_it, (size_t)last * 4, hipMemcpyDeviceToHost) != hipSuccess)
                throw fpldpc_error(FPLDPC_ERR_HIP, "DecodeTrial: hipMemcpy");
        } catch (const std::exception &e) {
            errs[r] = e.what();
            std::unique_lock<std::mutex> l(m);
            if (ready < R && ++ready == R) cv.notify_all();
        }
        (void)hipFree(d_llr);
        (void)hipFree(d_it);
    };
    std::vector<std::thread> th;
    for (int r = 1; r < R; r++) th.emplace_back(rank, r);
    rank(0);
    for (auto &t : th) t.join();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int r = 0; r < R; r++)
        if (!errs[r].empty()) throw fpldpc_error(FPLDPC_ERR_HIP, errs[r]);
    std::cout << sec << "  seconds" << std::endl;
    std::cout << n * (double)MaxPacket / sec << " bits per second for decoder" << std::endl;  // coded, as :189
    std::cout << (n - Decoder.rank()) * (double)MaxPacket / sec << " information bits per second" << std::endl;
    if (R > 1) std::cout << "DecodeTrial over " << R << " decoders (per decoder: " << n * (double)MaxPacket / sec / R
                         << " bits per second)" << std::endl;
    // Correctness record (no reference counterpart; the reference discards decode_fixpoint's return
    // value here): each rank's last launch, checked to repeat per 100-vector tile and across ranks;
    // vectors 0..99 printed (tests/test_gpu_perftest.py compares them with the oracle).
    for (int r = 0; r < R; r++)
        for (size_t i = 0; i < its[r].size(); i++)
            if (its[r][i] != its[0][i % 100]) throw fpldpc_error(FPLDPC_ERR_ARG, "DecodeTrial: iteration counts differ between tiles");
    const int shown = (int)std::min<size_t>(its[0].size(), 100);
    std::cout << "decode_fixpoint iterations (vectors 0-" << shown - 1 << "): ";
    for (int i = 0; i < shown; i++) std::cout << its[0][i] << ", ";
    std::cout << std::endl;
    return 0;
}

int EncodeTrial(char *info, int MaxPacket) {
    // :193-215: MaxPacket encodes of the same 248-byte stream with G_array_forward.txt -- here on
    // the device (fpldpc_encoder_encode, batches of up to 65536 frames), timed with HIP events.
    fpldpc_code_t c = array_code();
    auto Encoder = encoder_for("G_array_forward.txt", c);
    const int k = Encoder->info_length(), n = Encoder->length();
    std::vector<uint8_t> bits(k);
    fpldpc_compat::check(fpldpc_unpack_info_bytes(info, 248, k, bits.data()), "encode");
    const int B = std::max(1, std::min(MaxPacket, 65536));
    std::vector<uint8_t> u((size_t)B * k), cw((size_t)n), ref((size_t)n);
    for (int i = 0; i < B; i++) memcpy(&u[(size_t)i * k], bits.data(), k);
    uint8_t *d_u = nullptr, *d_cw = nullptr;
    if (hipMalloc((void **)&d_u, u.size()) != hipSuccess || hipMalloc((void **)&d_cw, (size_t)B * n) != hipSuccess)
        throw fpldpc_error(FPLDPC_ERR_HIP, "EncodeTrial: hipMalloc");
    (void)hipMemcpy(d_u, u.data(), u.size(), hipMemcpyHostToDevice);
    fpldpc_compat::check(fpldpc_encoder_encode(Encoder->handle(), d_u, 1, d_cw, nullptr), "encode");  // binds tables
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, nullptr);
    for (int done = 0; done < MaxPacket; done += B)
        fpldpc_compat::check(fpldpc_encoder_encode(Encoder->handle(), d_u, std::min(B, MaxPacket - done), d_cw, nullptr),
                             "encode");
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double sec = ms * 1e-3;
    (void)hipMemcpy(cw.data(), d_cw, n, hipMemcpyDeviceToHost);
    fpldpc_compat::check(fpldpc_encoder_encode_host(Encoder->handle(), bits.data(), 1, ref.data(), 1), "encode");
    if (cw != ref) throw fpldpc_error(FPLDPC_ERR_HIP, "EncodeTrial: device codeword differs from the host encoder");
    std::cout << sec << "  seconds" << std::endl;
    std::cout << 2209 * (double)MaxPacket / sec << " bits per second for encoder" << std::endl;
    (void)hipFree(d_u);
    (void)hipFree(d_cw);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    fpldpc_code_free(c);
    return 0;
}
