// ORACLE helper (test infrastructure): runs the reference's vendored kaldi-native-fbank on a raw
// float32 waveform and writes the fbank matrix. Options mirror runtime/onnxruntime/src/paraformer.cpp:21-31
// (dither 0, hamming, 25/10 ms, 80 bins, energy_floor 0). Built by oracle/Makefile into oracle/_ref/.
//   knf_fbank <in.f32 samples already x32768> <out.f32 [N,80]>
#include <cstdio>
#include <vector>

#include "kaldi-native-fbank/csrc/online-feature.h"

int main(int argc, char** argv) {
    if (argc != 3) { std::fprintf(stderr, "usage: knf_fbank in.f32 out.f32\n"); return 2; }
    std::FILE* fi = std::fopen(argv[1], "rb");
    if (!fi) return 3;
    std::vector<float> wav;
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, sizeof(float), 4096, fi)) > 0) wav.insert(wav.end(), buf, buf + n);
    std::fclose(fi);
    knf::FbankOptions opts;
    opts.frame_opts.dither = 0;
    opts.frame_opts.samp_freq = 16000;
    opts.frame_opts.window_type = "hamming";
    opts.frame_opts.frame_shift_ms = 10;
    opts.frame_opts.frame_length_ms = 25;
    opts.mel_opts.num_bins = 80;
    opts.energy_floor = 0;
    opts.mel_opts.debug_mel = false;
    knf::OnlineFbank fb(opts);
    fb.AcceptWaveform(16000, wav.data(), (int32_t)wav.size());
    fb.InputFinished();
    std::FILE* fo = std::fopen(argv[2], "wb");
    if (!fo) return 4;
    for (int32_t i = 0; i < fb.NumFramesReady(); ++i) std::fwrite(fb.GetFrame(i), sizeof(float), 80, fo);
    std::fclose(fo);
    return 0;
}
