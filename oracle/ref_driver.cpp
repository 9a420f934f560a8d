// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Our own command-line driver around the reference's UNMODIFIED sources, compiled in place from
// /root/reference (ArrayLDPC_Decoder.cpp, ArrayLDPC_Encoder.cpp, rngs.cpp, rvgs.cpp) by
// oracle/Makefile into oracle/_ref/ref_<dims>.  ref_wifi keeps the reference header as it is
// (WiFi (1944, 972) code, MAX_ITER 30, FRAC_WIDTH 4, WIDTH_MASK 0xff, ArrayLDPCMacro.h:17-39);
// ref_a47r5 / ref_a47r24 force-include the same header with the dimension enums substituted by
// oracle/ref_dims.sh (p47/r5: 30 it, mask 0xff; p47/r24: 50 it, mask 0x3f).  Used only to
// generate the golden fixtures under tests/golden/ (tests/golden/make_golden.py); never shipped.
//
// It replaces the Windows-only harness (PerfTest.cpp, Wrapper.cpp: windows.h /
// QueryPerformanceCounter) by re-stating the loops of ArrayLDPC_Debug_Wifi (PerfTest.cpp:23-140),
// ArrayLDPC_Debug (:217-316) and DecodeTrial (:148-192) here.
// The reference header first: glibc's <limits.h> defines an INT_WIDTH macro that collides
// with the reference's enum Precision (ArrayLDPCMacro.h:35), so <limits.h> is not included.
#include "ArrayLDPCMacro.h"
#include "rngs.h"
#include "rvgs.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <string>
#include <vector>
#include <unistd.h>
#ifndef PATH_MAX
#define PATH_MAX 4096
#endif

static FP_Decoder g_dec;  // large fixed-size members; static storage, zero-initialised
static const char *kRefDir = "/root/reference";
// PerfTest.cpp:33
static char g_info_stream[122] = "OMG  how long   dd   should this string be to make it 243";

static void die(const char *m) { fprintf(stderr, "ref_driver: %s\n", m); exit(2); }

struct Cwd {
    char old[PATH_MAX];
    explicit Cwd(const char *dir) { if (!getcwd(old, sizeof old) || chdir(dir) != 0) die("chdir"); }
    ~Cwd() { if (chdir(old) != 0) die("chdir back"); }
};

// Encoder + info bookkeeping exactly as PerfTest.cpp:54-96.
struct KatSetup {
    std::vector<int> cw;
    std::vector<int> info_idx;
    KatSetup() : cw(CWD_LENGTH), info_idx(INFO_LENGTH) {
        if (CWD_LENGTH != 1944 || INFO_LENGTH != 972) die("WiFi-only mode: use ref_wifi");
        Cwd d(kRefDir);
        static FP_Encoder enc((char *)"H_802.11_IndZerog.txt", 0);
        g_dec.setInfoBit(g_info_stream, 122);
        for (int i = 0; i < INFO_LENGTH; i++) info_idx[i] = enc.getInfoIndex(i);
        enc.encode(g_info_stream, 122);
        g_dec.setInfoIndex(info_idx.data());
        for (int i = 0; i < CWD_LENGTH; i++) cw[i] = enc.getCodeword(i);
        g_dec.ReadH();  // hard-coded "H_802.11_IndZero.txt" (ArrayLDPC_Decoder.cpp:646)
    }
};

static void read_h_from(const char *alist) {
    // ReadH opens "H_802.11_IndZero.txt" in the cwd; stage the requested alist under that name.
    char tmpl[] = "/tmp/ref_driver_XXXXXX";
    char *dir = mkdtemp(tmpl);
    if (!dir) die("mkdtemp");
    std::string link = std::string(dir) + "/H_802.11_IndZero.txt";
    char abs_path[PATH_MAX];
    if (!realpath(alist, abs_path)) die("realpath");
    if (symlink(abs_path, link.c_str()) != 0) die("symlink");
    {
        Cwd d(dir);
        g_dec.ReadH();
    }
    unlink(link.c_str());
    rmdir(dir);
}

int main(int argc, char **argv) {
    if (argc < 2) die("usage: ref_driver {kat_w|codeword|frames|sxor|decode} ...");
    std::string mode = argv[1];
    if (mode == "kat_w") {
        // kat_w EbN0 [max_frames] [checkpoint_every]: PerfTest.cpp:57-137 without cin.
        double EbN0_dB = atof(argv[2]);
        long max_frames = argc > 3 ? atol(argv[3]) : -1;
        long every = argc > 4 ? atol(argv[4]) : 0;
        KatSetup ks;
        double snr = 2 * pow(10.0, EbN0_dB / 10) * 0.5;
        double sigma = sqrt(1 / snr);
        int LLR_fp[CWD_LENGTH];
        double LLR[CWD_LENGTH];
        double biterror = 0, pckerror = 0, blkerror = 0;
        long Counter = 0;
        while (pckerror < 100 && (max_frames < 0 || Counter < max_frames)) {
            for (int i = 0; i < CWD_LENGTH; i++) {
                LLR[i] = 2 * snr * (1 - 2 * ks.cw[i] + Normal(0, sigma));
                LLR_fp[i] = int(LLR[i] * (1 << FRAC_WIDTH));
            }
            g_dec.setState(PCV);
            g_dec.decode_general_fp(LLR_fp);
            g_dec.resetBER();
            blkerror = g_dec.calculateBER();
            if (blkerror > 0) pckerror++;
            biterror += blkerror;
            Counter++;
            if (every > 0 && Counter % every == 0)
                printf("checkpoint %ld %.0f %.0f\n", Counter, biterror, pckerror);
        }
        printf("%.0f %.0f %ld\n", biterror, pckerror, Counter);
        printf(" FER: %g BER: %g\n", pckerror / Counter, biterror / Counter / CWD_LENGTH);
        return 0;
    }
    if (mode == "codeword") {
        KatSetup ks;
        for (int i = 0; i < CWD_LENGTH; i++) printf("%d%c", ks.cw[i], i + 1 < CWD_LENGTH ? ' ' : '\n');
        for (int i = 0; i < INFO_LENGTH; i++) printf("%d%c", ks.info_idx[i], i + 1 < INFO_LENGTH ? ' ' : '\n');
        return 0;
    }
    if (mode == "frames") {
        // frames EbN0 nframes skip_frames use_cw out.bin : per frame int32 LLR[N], iter, post[N]
        if (argc < 7) die("frames EbN0 nframes skip use_cw out");
        double EbN0_dB = atof(argv[2]);
        long nframes = atol(argv[3]), skip = atol(argv[4]);
        int use_cw = atoi(argv[5]);
        KatSetup ks;
        double snr = 2 * pow(10.0, EbN0_dB / 10) * 0.5;
        double sigma = sqrt(1 / snr);
        for (long i = 0; i < skip * CWD_LENGTH; i++) Random();
        FILE *f = fopen(argv[6], "wb");
        if (!f) die("open out");
        int LLR_fp[CWD_LENGTH], post[CWD_LENGTH];
        for (long fr = 0; fr < nframes; fr++) {
            for (int i = 0; i < CWD_LENGTH; i++) {
                double L = 2 * snr * (1 - 2 * (use_cw ? ks.cw[i] : 0) + Normal(0, sigma));
                LLR_fp[i] = int(L * (1 << FRAC_WIDTH));
            }
            g_dec.setState(PCV);
            int it = g_dec.decode_general_fp(LLR_fp);
            for (int i = 0; i < CWD_LENGTH; i++) post[i] = g_dec.getPost_fp(i);
            fwrite(LLR_fp, sizeof(int), CWD_LENGTH, f);
            fwrite(&it, sizeof(int), 1, f);
            fwrite(post, sizeof(int), CWD_LENGTH, f);
        }
        fclose(f);
        return 0;
    }
    if (mode == "float_frames") {
        // float_frames EbN0 nframes skip use_cw out.bin : the floating-point decoder
        // FP_Decoder::decode_general (ArrayLDPC_Decoder.cpp:735-933) on unquantised LLRs
        // LLR = 2*snr*(1 - 2c + Normal(0, sigma)) (PerfTest.cpp:108-110); per frame
        // double LLR[N], int iter, double post[N] (getPost, ArrayLDPCMacro.h:149).
        if (argc < 7) die("float_frames EbN0 nframes skip use_cw out");
        double EbN0_dB = atof(argv[2]);
        long nframes = atol(argv[3]), skip = atol(argv[4]);
        int use_cw = atoi(argv[5]);
        KatSetup ks;
        double snr = 2 * pow(10.0, EbN0_dB / 10) * 0.5;
        double sigma = sqrt(1 / snr);
        for (long i = 0; i < skip * CWD_LENGTH; i++) Random();
        FILE *f = fopen(argv[6], "wb");
        if (!f) die("open out");
        double LLR[CWD_LENGTH], post[CWD_LENGTH];
        for (long fr = 0; fr < nframes; fr++) {
            for (int i = 0; i < CWD_LENGTH; i++) LLR[i] = 2 * snr * (1 - 2 * (use_cw ? ks.cw[i] : 0) + Normal(0, sigma));
            int it = g_dec.decode_general(LLR);
            for (int i = 0; i < CWD_LENGTH; i++) post[i] = g_dec.getPost(i);
            fwrite(LLR, sizeof(double), CWD_LENGTH, f);
            fwrite(&it, sizeof(int), 1, f);
            fwrite(post, sizeof(double), CWD_LENGTH, f);
        }
        fclose(f);
        return 0;
    }
    if (mode == "sxor_f64") {
        // sxor_f64 in.bin count out.bin : pairs of doubles -> FP_Decoder::sxor(double, double)
        // (ArrayLDPC_Decoder.cpp:724-732)
        FILE *fi = fopen(argv[2], "rb");
        long cnt = atol(argv[3]);
        FILE *fo = fopen(argv[4], "wb");
        if (!fi || !fo) die("open");
        for (long i = 0; i < cnt; i++) {
            double xy[2];
            if (fread(xy, sizeof(double), 2, fi) != 2) die("short in");
            double r = g_dec.sxor(xy[0], xy[1]);
            fwrite(&r, sizeof(double), 1, fo);
        }
        fclose(fi);
        fclose(fo);
        return 0;
    }
    if (mode == "sxor") {
        // sxor lo hi out.bin : int32 table [x][y] of FP_Decoder::sxor (FRAC 4, mask 0xff)
        int lo = atoi(argv[2]), hi = atoi(argv[3]);
        FILE *f = fopen(argv[4], "wb");
        if (!f) die("open out");
        std::vector<int> row(hi - lo + 1);
        for (int x = lo; x <= hi; x++) {
            for (int y = lo; y <= hi; y++) row[y - lo] = g_dec.sxor(x, y);
            fwrite(row.data(), sizeof(int), row.size(), f);
        }
        fclose(f);
        return 0;
    }
    if (mode == "rng") {
        // rng n : TestRandom()'s verdict (rngs.cpp:154-180), then from the default seed 123456789
        // (rngs.cpp:45) n Lehmer states, then n Normal(0,1) values (rvgs.cpp:152-181) as %a.
        long n = argc > 2 ? atol(argv[2]) : 16;
        TestRandom();
        SelectStream(0);
        PutSeed(123456789);
        for (long i = 0; i < n; i++) {
            Random();
            long s;
            GetSeed(&s);
            printf("state %ld\n", s);
        }
        PutSeed(123456789);
        for (long i = 0; i < n; i++) printf("normal %a\n", Normal(0, 1));
        PutSeed(1);
        for (long i = 0; i < 10000; i++) Random();
        long s;
        GetSeed(&s);
        printf("seed1_after_10000 %ld\n", s);
        return 0;
    }
    if (mode == "decode") {
        // decode alist llr.bin nframes out.bin [fixpoint] : llr int32 [nframes][CWD_LENGTH];
        // out per frame int32 iter, post[N] (getPost_fp), hard[N] (DecodedCodeword).
        // fixpoint = 1: setState(PCV) + decode_fixpoint (ArrayLDPC_Decoder.cpp:422-639, ROM-addressed,
        // with the hardDecision pre-check :443-450); else decode_general_fp (:18-171) on the alist.
        if (argc < 6) die("decode alist llr nframes out [fixpoint]");
        read_h_from(argv[2]);
        long nframes = atol(argv[4]);
        int fixpoint = argc > 6 ? atoi(argv[6]) : 0;
        FILE *fi = fopen(argv[3], "rb");
        FILE *fo = fopen(argv[5], "wb");
        if (!fi || !fo) die("open");
        int LLR_fp[CWD_LENGTH], post[CWD_LENGTH];
        for (long fr = 0; fr < nframes; fr++) {
            if (fread(LLR_fp, sizeof(int), CWD_LENGTH, fi) != (size_t)CWD_LENGTH) die("short llr");
            g_dec.setState(PCV);
            int it = fixpoint ? g_dec.decode_fixpoint(LLR_fp) : g_dec.decode_general_fp(LLR_fp);
            for (int i = 0; i < CWD_LENGTH; i++) post[i] = g_dec.getPost_fp(i);
            fwrite(&it, sizeof(int), 1, fo);
            fwrite(post, sizeof(int), CWD_LENGTH, fo);
            fwrite(g_dec.DecodedCodeword, sizeof(int), CWD_LENGTH, fo);
        }
        fclose(fi);
        fclose(fo);
        return 0;
    }
    if (mode == "fsm") {
        // fsm alist llr.bin nframes out.bin flags : decode_fixpoint per frame, setState(PCV) before
        // frame f only when flags[f] == '1' (the FSM of ArrayLDPC_Decoder.cpp:443-488, :621-630 across
        // calls); out per frame int32 iter, FSM state after the call, post[N], hard[N], and the edge
        // RAM EdgeRAM[k].BRAM_fp[c] (k < CHK_DEG, c < NUM_CHK) the call left.
        if (argc < 7) die("fsm alist llr nframes out flags");
        read_h_from(argv[2]);
        long nframes = atol(argv[4]);
        const char *flags = argv[6];
        if ((long)strlen(flags) != nframes) die("fsm: one flag per frame");
        FILE *fi = fopen(argv[3], "rb");
        FILE *fo = fopen(argv[5], "wb");
        if (!fi || !fo) die("open");
        int LLR_fp[CWD_LENGTH], post[CWD_LENGTH];
        for (long fr = 0; fr < nframes; fr++) {
            if (fread(LLR_fp, sizeof(int), CWD_LENGTH, fi) != (size_t)CWD_LENGTH) die("short llr");
            if (flags[fr] == '1') g_dec.setState(PCV);
            int it = g_dec.decode_fixpoint(LLR_fp);
            int st = g_dec.getState();
            for (int i = 0; i < CWD_LENGTH; i++) post[i] = g_dec.getPost_fp(i);
            fwrite(&it, sizeof(int), 1, fo);
            fwrite(&st, sizeof(int), 1, fo);
            fwrite(post, sizeof(int), CWD_LENGTH, fo);
            fwrite(g_dec.DecodedCodeword, sizeof(int), CWD_LENGTH, fo);
            for (int k = 0; k < CHK_DEG; k++) fwrite(g_dec.EdgeRAM[k].BRAM_fp, sizeof(int), NUM_CHK, fo);
        }
        fclose(fi);
        fclose(fo);
        return 0;
    }
    if (mode == "dims") {
        // the compile-time parameters this binary was built with (ArrayLDPCMacro.h:17-39, :175)
        printf("NUM_VAR %d NUM_CHK %d NUM_CGRP %d NUM_VGRP %d CHK_DEG %d VAR_DEG %d P %d INFO_LENGTH %d "
               "CWD_LENGTH %d MAX_ITER %d WIDTH_MASK %d FRAC_WIDTH %d RAM_DEPTH %d\n",
               (int)NUM_VAR, (int)NUM_CHK, (int)NUM_CGRP, (int)NUM_VGRP, (int)CHK_DEG, (int)VAR_DEG, (int)P,
               (int)INFO_LENGTH, (int)CWD_LENGTH, (int)MAX_ITER, (int)WIDTH_MASK, (int)FRAC_WIDTH, (int)RAM_DEPTH);
        printf("rate %a\n", g_dec.getRate());
        return 0;
    }
    if (mode == "chan") {
        // chan EbN0 rate nframes skip out.bin : all-zero-codeword BPSK/AWGN LLRs of the benchmark
        // loops (PerfTest.cpp:164-170, 587-590): LLR = 2*snr*(1 + Normal(0, sigma)),
        // LLR_fp = int(LLR * 2^FRAC), snr = 2*10^(EbN0/10)*rate; rate <= 0 means getRate()
        // (ROM::CodeRate, ArrayLDPCMacro.h:60).  Draws start after skip*CWD_LENGTH Random() calls.
        if (argc < 7) die("chan EbN0 rate nframes skip out");
        double EbN0_dB = atof(argv[2]), rate = atof(argv[3]);
        long nframes = atol(argv[4]), skip = atol(argv[5]);
        if (rate <= 0) rate = g_dec.getRate();
        double snr = 2 * pow(10.0, EbN0_dB / 10) * rate;
        double sigma = sqrt(1 / snr);
        for (long i = 0; i < skip * CWD_LENGTH; i++) Random();
        FILE *f = fopen(argv[6], "wb");
        if (!f) die("open out");
        int LLR_fp[CWD_LENGTH];
        for (long fr = 0; fr < nframes; fr++) {
            for (int i = 0; i < CWD_LENGTH; i++) LLR_fp[i] = int(2 * snr * (1 + Normal(0, sigma)) * (1 << FRAC_WIDTH));
            fwrite(LLR_fp, sizeof(int), CWD_LENGTH, f);
        }
        fclose(f);
        return 0;
    }
    if (mode == "decodetrial") {
        // decodetrial EbN0 MaxPacket out.bin : DecodeTrial (PerfTest.cpp:148-192) without the
        // timer: 100 all-zero-codeword frames at getRate(), then decode_fixpoint on frame i % 100
        // for i < MaxPacket.  out per packet: int32 return value, hard[N] (DecodedCodeword).
        if (argc < 5) die("decodetrial EbN0 MaxPacket out");
        double EbN0_dB = atof(argv[2]);
        long max_packet = atol(argv[3]);
        static int LLR_fp[100][CWD_LENGTH];
        double snr = 2 * pow(10.0, EbN0_dB / 10) * g_dec.getRate();
        double sigma = sqrt(1 / snr);
        for (int j = 0; j < 100; j++)
            for (int i = 0; i < CWD_LENGTH; i++) LLR_fp[j][i] = int(2 * snr * (1 + Normal(0, sigma)) * (1 << FRAC_WIDTH));
        FILE *f = fopen(argv[4], "wb");
        if (!f) die("open out");
        for (long i = 0; i < max_packet; i++) {
            g_dec.setState(PCV);
            int it = g_dec.decode_fixpoint(LLR_fp[i % 100]);
            fwrite(&it, sizeof(int), 1, f);
            fwrite(g_dec.DecodedCodeword, sizeof(int), CWD_LENGTH, f);
        }
        fclose(f);
        return 0;
    }
    if (mode == "kat_a") {
        // kat_a EbN0 info.bin [checkpoint_every] : ArrayLDPC_Debug (PerfTest.cpp:217-316) with
        // EbN0 as an argument.  info.bin holds the 248-byte InfoStream literal of :221-224
        // (extracted by make_golden.py).  FP_Encoder("G_array_forward.txt") needs G_mlist
        // [972][1078] (ref_a47r5).  Prints "bit_errors frame_errors frames" and the FER/BER line.
        if (CWD_LENGTH != 2209 || INFO_LENGTH != 1978) die("kat_a needs ref_a47r5");
        if (argc < 4) die("kat_a EbN0 info.bin [every]");
        double EbN0_dB = atof(argv[2]);
        long every = argc > 4 ? atol(argv[4]) : 0;
        static char InfoStream[248];
        FILE *fi = fopen(argv[3], "rb");
        if (!fi || fread(InfoStream, 1, 248, fi) != 248) die("info.bin");
        fclose(fi);
        static FP_Encoder *enc;
        {
            std::string codes = std::string(kRefDir) + "/codes";
            Cwd d(codes.c_str());
            enc = new FP_Encoder((char *)"G_array_forward.txt", 0);
        }
        double snr = 2 * pow(10.0, EbN0_dB / 10) * g_dec.getRate();
        double sigma = sqrt(1 / snr);
        static int info_indx[INFO_LENGTH];
        g_dec.setInfoBit(InfoStream, 248);
        for (int i = 0; i < INFO_LENGTH; i++) info_indx[i] = enc->getInfoIndex(i);
        g_dec.setInfoIndex(info_indx);
        double biterror = 0, pckerror = 0, blkerror = 0;
        long Counter = 0;
        int LLR_fp[CWD_LENGTH];
        while (pckerror < 100) {
            enc->encode(InfoStream, 248);
            for (int i = 0; i < CWD_LENGTH; i++)
                LLR_fp[i] = int(2 * snr * (1 - 2 * enc->getCodeword(i) + Normal(0, sigma)) * (1 << FRAC_WIDTH));
            g_dec.setState(PCV);
            g_dec.decode_fixpoint(LLR_fp);
            g_dec.resetBER();
            blkerror = g_dec.calculateBER();
            if (blkerror > 0) pckerror++;
            biterror += blkerror;
            Counter++;
            if (every > 0 && Counter % every == 0) printf("checkpoint %ld %.0f %.0f\n", Counter, biterror, pckerror);
        }
        printf("%.0f %.0f %ld\n", biterror, pckerror, Counter);
        printf(" FER: %g BER: %g\n", pckerror / Counter, biterror / Counter / CWD_LENGTH);
        return 0;
    }
    die("unknown mode");
}
