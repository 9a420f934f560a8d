// fpldpc_perftest -- command-line driver of the PerfTest.h functions (fpldpc_compat.hpp), the
// counterpart of the reference's Wrapper.cpp main (Wrapper.cpp:17-101), non-interactive.
//   fpldpc_perftest wifi [EbN0]          ArrayLDPC_Debug_Wifi   (stdin prompt when EbN0 is omitted)
//   fpldpc_perftest array                ArrayLDPC_Debug        (4.5 dB, decode_fixpoint)
//   fpldpc_perftest shorten LEN          ArrayLDPC_Debug_Shorten
//   fpldpc_perftest decode_trial EbN0 N  DecodeTrial
//   fpldpc_perftest encode_trial N       EncodeTrial
//   fpldpc_perftest perftest db0 db1 step FILE   ArrayLDPC_PerfTest
//   fpldpc_perftest timetrial db N FILE          ArrayLDPC_TimeTrial
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "fpldpc_compat.hpp"

int main(int argc, char **argv) {
    if (argc < 2) {
        std::cerr << "usage: fpldpc_perftest {wifi|array|shorten|decode_trial|encode_trial|perftest|timetrial} ...\n";
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
        if (m == "timetrial" && argc > 4) return ArrayLDPC_TimeTrial(atof(argv[2]), atoi(argv[3]), argv[4]);
    } catch (const fpldpc_error &e) {
        std::cerr << "fpldpc_perftest: " << e.what() << "\n";
        return 1;
    }
    std::cerr << "fpldpc_perftest: bad arguments\n";
    return 2;
}
