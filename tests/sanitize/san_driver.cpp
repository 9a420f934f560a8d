// san_driver.cpp -- host-side code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5,
// "Race detection / sanitizers").  Built by tests/sanitize/Makefile from the library's host-only
// translation units (fpldpc_code.cpp, fpldpc_channel.cpp, fpldpc_encoder.cpp) and the oracle
// restatement (oracle/fpldpc_oracle.c), with no GPU code: the device kernels cannot run under GPU
// sanitizers on this pool.  It drives the paths where the reference has its memory hazards --
// function-static decoder state (ArrayLDPC_Decoder.cpp:21-37) becomes per-object state here, and
// the unchecked ReadH parse (:642-674) becomes a validating alist parser that must reject
// malformed input instead of reading out of bounds.  Exit 0 = every check passed; the sanitizers
// abort on the first report (-fno-sanitize-recover).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fpldpc.h"
#include "fpldpc_oracle.h"

static int failures = 0;
#define CHECK(cond)                                                        \
    do {                                                                   \
        if (!(cond)) {                                                     \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                    \
        }                                                                  \
    } while (0)

static std::string alist_text(fpldpc_code_t c) {
    size_t len = 0;
    CHECK(fpldpc_code_write_alist(c, nullptr, 0, &len) == FPLDPC_OK || len > 0);
    std::string s(len + 1, '\0');
    CHECK(fpldpc_code_write_alist(c, &s[0], s.size(), &len) == FPLDPC_OK);
    s.resize(len);
    return s;
}

// One code: alist round trip, hostile variants of its text, the host encoder and the oracle.
static void exercise(fpldpc_code_t c, const char *name, bool decode) {
    int32_t d[8];
    CHECK(fpldpc_code_dims(c, d) == FPLDPC_OK);
    const int n = d[0], m = d[1];
    const std::string text = alist_text(c);
    fpldpc_code_t c2 = nullptr;
    CHECK(fpldpc_code_parse_alist(text.data(), text.size(), &c2) == FPLDPC_OK);
    CHECK(alist_text(c2) == text);
    fpldpc_code_free(c2);

    // truncations at many points, and single tokens replaced by hostile values: every one must be
    // rejected (or, for a harmless edit, accepted) without an out-of-bounds access
    int rejected = 0, tried = 0;
    for (size_t cut = 0; cut < text.size(); cut += 1 + text.size() / 61) {
        fpldpc_code_t t = nullptr;
        const int st = fpldpc_code_parse_alist(text.data(), cut, &t);
        rejected += st != FPLDPC_OK;
        ++tried;
        if (st == FPLDPC_OK) fpldpc_code_free(t);
    }
    CHECK(rejected == tried);  // every strict prefix is incomplete
    const char *evil[] = {"-1", "0", "99999999", "2147483647", "x", "65536", "-7"};
    size_t pos = 0;
    for (int i = 0; i < 40; ++i) {
        pos = text.find_first_of("0123456789", pos + 1 + text.size() / 41);
        if (pos == std::string::npos) break;
        const size_t end = text.find_first_not_of("0123456789", pos);
        std::string bad = text.substr(0, pos) + evil[i % 7] + text.substr(end);
        fpldpc_code_t t = nullptr;
        if (fpldpc_code_parse_alist(bad.data(), bad.size(), &t) == FPLDPC_OK) fpldpc_code_free(t);
        pos = end;
    }
    fpldpc_code_t none = nullptr;
    CHECK(fpldpc_code_load_alist("/nonexistent/H.txt", &none) == FPLDPC_ERR_IO);

    // host encoder: every codeword satisfies H; info bytes unpack
    fpldpc_encoder_t enc = nullptr;
    CHECK(fpldpc_encoder_from_code(c, &enc) == FPLDPC_OK);
    int32_t ed[3];
    CHECK(fpldpc_encoder_dims(enc, ed) == FPLDPC_OK && ed[0] == n);
    const int k = ed[1], B = 6;
    std::vector<uint8_t> info((size_t)B * k), cw((size_t)B * n);
    uint32_t x = 12345;
    for (auto &b : info) b = (x = x * 1103515245u + 12345u) >> 31;
    CHECK(fpldpc_encoder_encode_host(enc, info.data(), B, cw.data(), 3) == FPLDPC_OK);
    for (int f = 0; f < B; ++f) CHECK(fpldpc_code_syndrome_host(c, &cw[(size_t)f * n]) == 0);
    std::vector<int32_t> ii(k), pi(n - k);
    CHECK(fpldpc_encoder_info_index(enc, ii.data(), pi.data()) == FPLDPC_OK);
    std::vector<char> bytes((k + 7) / 8, 'Z');
    std::vector<uint8_t> bits(k);
    CHECK(fpldpc_unpack_info_bytes(bytes.data(), (int)bytes.size(), k, bits.data()) == FPLDPC_OK);
    fpldpc_encoder_free(enc);

    // channel (threaded skip-ahead) against the oracle's serial restatement, all output types
    const int F = 3;
    const double snr = 2 * std::pow(10.0, 0.2) * 0.5, sigma = std::sqrt(1 / snr);
    std::vector<int32_t> l32((size_t)F * n), o32((size_t)F * n);
    std::vector<int16_t> l16((size_t)F * n);
    std::vector<double> l64((size_t)F * n);
    CHECK(fpldpc_channel_llr_host(123456789, 5, F, n, snr, sigma, 4, cw.data(), l32.data(), FPLDPC_LLR_I32, 3) == 0);
    CHECK(fpldpc_channel_llr_host(123456789, 5, F, n, snr, sigma, 4, cw.data(), l16.data(), FPLDPC_LLR_I16, 2) == 0);
    CHECK(fpldpc_channel_llr_host(123456789, 5, F, n, snr, sigma, 4, cw.data(), l64.data(), FPLDPC_LLR_F64, 4) == 0);
    orc_gen_llr(123456789, 5, F, n, snr, sigma, 4, cw.data(), o32.data(), 1);
    CHECK(l32 == o32);
    for (size_t i = 0; i < l16.size(); ++i) CHECK(l16[i] == l32[i]);

    if (decode) {  // the oracle decoders on the same frames (alist through a file, as ReadH)
        char path[] = "/tmp/fpldpc_san_XXXXXX";
        const int fd = mkstemp(path);
        CHECK(fd >= 0);
        FILE *fp = fdopen(fd, "w");
        fwrite(text.data(), 1, text.size(), fp);
        fclose(fp);
        orc_code oc;
        CHECK(orc_code_load_alist(path, &oc) == 0);
        remove(path);
        std::vector<int32_t> its(F), post((size_t)F * n);
        std::vector<uint8_t> ok(F), hard((size_t)F * n);
        orc_decode_batch(&oc, l16.data(), 1, F, 8, orc_constant(4), 0xff, 0, 3, its.data(), ok.data(), hard.data(),
                         post.data());
        std::vector<int32_t> its2(F);
        orc_decode_batch(&oc, l32.data(), 0, F, 8, orc_constant(4), 0x3f, 1, 1, its2.data(), nullptr, nullptr, nullptr);
        for (int f = 0; f < F; ++f) CHECK(its[f] >= 1 && its[f] <= 8 && its2[f] >= 0 && its2[f] <= 8);
        std::vector<double> fpost(n);
        std::vector<uint8_t> fhard(n);
        int syn = 0;
        const int fit = orc_decode_float(&oc, l64.data(), 5, fpost.data(), fhard.data(), &syn);
        CHECK(fit >= 1 && fit <= 5);
        orc_code_free(&oc);
    }
    printf("%s: n=%d m=%d k=%d, %d truncations rejected\n", name, n, m, k, rejected);
}

int main() {
    CHECK(orc_test_random() == 1);
    std::vector<int32_t> tab(41 * 41);
    orc_sxor_table(-20, 20, orc_constant(4), 0xff, tab.data());
    CHECK(tab[20 * 41 + 20] == orc_sxor(0, 0, orc_constant(4), 0xff));
    fpldpc_code_t a = nullptr, r = nullptr, w = nullptr, bad = nullptr;
    CHECK(fpldpc_code_array(47, 5, 1, &a) == FPLDPC_OK);
    CHECK(fpldpc_code_array(47, 24, 1, &r) == FPLDPC_OK);
    CHECK(fpldpc_code_wifi_1944_r12(&w) == FPLDPC_OK);
    CHECK(fpldpc_code_array(4, 5, 1, &bad) != FPLDPC_OK);  // p not prime
    exercise(a, "array p47 r5", true);
    exercise(w, "802.11n 1944", true);
    exercise(r, "array p47 r24", false);
    fpldpc_code_free(a);
    fpldpc_code_free(r);
    fpldpc_code_free(w);
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("sanitizer driver: all checks passed\n");
    return 0;
}
