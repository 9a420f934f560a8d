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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include <cmath>
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
        if (m == "timetrial" && argc > 4) return ArrayLDPC_TimeTrial(atof(argv[2]), atoi(argv[3]), argv[4]);
    } catch (const fpldpc_error &e) {
        std::cerr << "fpldpc_perftest: " << e.what() << "\n";
        return 1;
    }
    std::cerr << "fpldpc_perftest: bad arguments\n";
    return 2;
}
