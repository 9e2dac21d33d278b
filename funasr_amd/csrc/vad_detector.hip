// FSMN-VAD detection state machine (include/pfm.h, pfm_vad_detector_*): host C++ only (no device code), built
// into libpfm_hip.so with the rest of csrc/ and, for the host sanitizer test (tests/test_host_sanitize.py), alone
// with g++ -fsanitize=address,undefined.
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <vector>

#include "pfm.h"

int pfm_fail(int code, const char* msg);   // pfm_api.hip: sets pfm_last_error()

// ============================================================================================
// FSMN-VAD detection state machine (include/pfm.h, pfm_vad_detector_*): host code, the per-frame
// decision loop of E2EVadModel (fsmn_vad_streaming/model.py:303-916) over the posteriors pfm_vad_run
// produced and the frame decibels. Values are kept with absolute frame indices (the reference drops
// consumed frames from the front of its arrays and indexes relative to the drop count: same element).
// ============================================================================================
namespace {
enum { VS_START = 1, VS_SPEECH = 2, VS_END = 3 };
enum { FS_INVALID = -1, FS_SIL = 0, FS_SPEECH = 1 };
enum { CH_S2S = 0, CH_SP2SIL = 1, CH_SIL2SIL = 2, CH_SIL2SP = 3, CH_INVALID = 5 };
struct VadSeg { int start_ms, end_ms; bool has_start, has_end; };
}  // namespace

struct pfm_vad_detector {
    pfm_vad_opts o;
    // WindowDetector (model.py:159-241)
    int win = 0, s2p = 0, p2s = 0, wpos = 0, wsum = 0, wpre = FS_SIL;
    std::vector<int> wstate;
    std::vector<double> db;
    std::vector<float> ps;
    int data_buf_start = 0, frm_cnt = 0, latest_speech = 0, latest_sil = -1, cont_sil = 0, state = VS_START;
    int conf_start = -1, conf_end = -1, n_end = 0, last_drop = 0, out_offset = 0;
    double noise_db = -100.0;
    bool next_seg = true;
    std::vector<VadSeg> out;

    void win_reset() { wpos = 0; wsum = 0; std::fill(wstate.begin(), wstate.end(), 0); wpre = FS_SIL; }
    int win_detect(int fs) {
        if (fs != FS_SPEECH && fs != FS_SIL) return CH_INVALID;
        const int cur = fs == FS_SPEECH ? 1 : 0;
        wsum += cur - wstate[wpos];
        wstate[wpos] = cur;
        wpos = (wpos + 1) % win;
        if (wpre == FS_SIL && wsum >= s2p) { wpre = FS_SPEECH; return CH_SIL2SP; }
        if (wpre == FS_SPEECH && wsum <= p2s) { wpre = FS_SIL; return CH_SP2SIL; }
        return wpre == FS_SIL ? CH_SIL2SIL : CH_S2S;
    }
    int latency() const { return win + (o.do_extend ? (int)((double)o.lookback_time_start_point / o.frame_in_ms) : 0); }
    void pop_till(int f) { if (data_buf_start < f) data_buf_start = f; }
    void pop_to_output(int start, int cnt, bool first_is_start, bool last_is_end) {
        pop_till(start);
        if (out.empty() || first_is_start) out.push_back({start * o.frame_in_ms, start * o.frame_in_ms, false, false});
        VadSeg& s = out.back();
        data_buf_start += cnt;
        s.end_ms = (start + cnt) * o.frame_in_ms;
        if (first_is_start) s.has_start = true;
        if (last_is_end) s.has_end = true;
    }
    void on_silence(int f) { latest_sil = f; if (state == VS_START) pop_till(f); }
    void on_voice(int f) { latest_speech = f; pop_to_output(f, 1, false, false); }
    void on_voice_start(int f, bool fake) {
        if (conf_start == -1) conf_start = f;
        if (!fake && state == VS_START) pop_to_output(conf_start, 1, true, false);
    }
    void on_voice_end(int f, bool fake) {
        for (int t = latest_speech + 1; t < f; ++t) on_voice(t);
        if (conf_end == -1) conf_end = f;
        if (!fake) pop_to_output(conf_end, 1, false, true);
        ++n_end;
    }
    void maybe_end_if_last(bool fin, int idx) { if (fin) { on_voice_end(idx, false); state = VS_END; } }
    int reset_detection() {
        cont_sil = 0; latest_speech = 0; latest_sil = -1; conf_start = -1; conf_end = -1; state = VS_START;
        win_reset();
        if (!out.empty()) {
            if (!out.back().has_end) return -1;
            last_drop = (int)((double)out.back().end_ms / o.frame_in_ms);
        }
        return 0;
    }
    int frame_state(int t) {
        const double d = db[t];
        const double snr = d - noise_db;
        if (d < o.decibel_thres) {
            int rc = detect_one(FS_SIL, t - last_drop, false);
            if (rc) return -100;
            return FS_SIL;
        }
        const double s = (double)ps[t];
        const double noise_prob = std::log(s) * o.speech_2_noise_ratio;
        const double speech_prob = std::log(1.0 - s);
        if (std::exp(speech_prob) >= std::exp(noise_prob) + o.speech_noise_thres) {
            if (snr >= o.snr_thres && d >= o.decibel_thres) return FS_SPEECH;
            return FS_SIL;
        }
        if (noise_db < -99.9) noise_db = d;
        else noise_db = (d + noise_db * (o.noise_frame_num_used_for_snr - 1)) / o.noise_frame_num_used_for_snr;
        return FS_SIL;
    }
    int detect_one(int fs, int idx, bool fin) {
        int tmp = FS_INVALID;
        if (fs == FS_SPEECH) tmp = std::fabs(1.0) > o.fe_prior_thres ? FS_SPEECH : FS_SIL;
        else if (fs == FS_SIL) tmp = FS_SIL;
        const int ch = win_detect(tmp);
        const double max_seg = (double)o.max_single_segment_time / o.frame_in_ms;
        const int max_end_sil = o.max_end_silence_time - o.speech_to_sil_time_thres;
        if (ch == CH_SIL2SP) {
            cont_sil = 0;
            if (state == VS_START) {
                const int start = std::max(data_buf_start, idx - latency());
                on_voice_start(start, false);
                state = VS_SPEECH;
                for (int t = start + 1; t < idx + 1; ++t) on_voice(t);
            } else if (state == VS_SPEECH) {
                for (int t = latest_speech + 1; t < idx; ++t) on_voice(t);
                if (idx - conf_start + 1 > max_seg) { on_voice_end(idx, false); state = VS_END; }
                else if (!fin) on_voice(idx);
                else maybe_end_if_last(fin, idx);
            }
        } else if (ch == CH_SP2SIL || ch == CH_S2S) {
            cont_sil = 0;
            if (state == VS_SPEECH) {
                if (idx - conf_start + 1 > max_seg) { on_voice_end(idx, false); state = VS_END; }
                else if (!fin) on_voice(idx);
                else maybe_end_if_last(fin, idx);
            }
        } else if (ch == CH_SIL2SIL) {
            ++cont_sil;
            if (state == VS_START) {
                if ((o.detect_mode == 0 && cont_sil * o.frame_in_ms > o.max_start_silence_time) || (fin && n_end == 0)) {
                    for (int t = latest_sil + 1; t < idx; ++t) on_silence(t);
                    on_voice_start(0, true);
                    on_voice_end(0, true);
                    state = VS_END;
                } else if (idx >= latency()) {
                    on_silence(idx - latency());
                }
            } else if (state == VS_SPEECH) {
                if (cont_sil * o.frame_in_ms >= max_end_sil) {
                    int look = (int)((double)max_end_sil / o.frame_in_ms);
                    if (o.do_extend) {
                        look -= (int)((double)o.lookahead_time_end_point / o.frame_in_ms);
                        look -= 1;
                        look = std::max(0, look);
                    }
                    on_voice_end(idx - look, false);
                    state = VS_END;
                } else if (idx - conf_start + 1 > max_seg) {
                    on_voice_end(idx, false);
                    state = VS_END;
                } else if (o.do_extend && !fin) {
                    if (cont_sil <= (int)((double)o.lookahead_time_end_point / o.frame_in_ms)) on_voice(idx);
                } else {
                    maybe_end_if_last(fin, idx);
                }
            }
        }
        if (state == VS_END && o.detect_mode == 1) return reset_detection();
        return 0;
    }
};

extern "C" {

void pfm_vad_opts_default(pfm_vad_opts* o) {
    o->detect_mode = 1; o->max_end_silence_time = 800; o->max_start_silence_time = 3000; o->window_size_ms = 200;
    o->sil_to_speech_time_thres = 150; o->speech_to_sil_time_thres = 150; o->do_extend = 1;
    o->lookback_time_start_point = 200; o->lookahead_time_end_point = 100; o->max_single_segment_time = 60000;
    o->noise_frame_num_used_for_snr = 100; o->frame_in_ms = 10;
    o->speech_2_noise_ratio = 1.0; o->snr_thres = -100.0; o->decibel_thres = -100.0; o->speech_noise_thres = 0.6;
    o->fe_prior_thres = 1e-4;
}

int pfm_vad_detector_create(const pfm_vad_opts* o, pfm_vad_detector** out) {
    if (!o || !out) return pfm_fail(PFM_E_ARG, "pfm_vad_detector_create: null argument");
    *out = nullptr;
    if (o->frame_in_ms < 1 || o->window_size_ms < o->frame_in_ms || o->noise_frame_num_used_for_snr < 1)
        return pfm_fail(PFM_E_ARG, "pfm_vad_detector_create: bad options");
    std::unique_ptr<pfm_vad_detector> d(new pfm_vad_detector());
    d->o = *o;
    d->win = o->window_size_ms / o->frame_in_ms;
    d->s2p = o->sil_to_speech_time_thres / o->frame_in_ms;
    d->p2s = o->speech_to_sil_time_thres / o->frame_in_ms;
    d->wstate.assign(d->win, 0);
    *out = d.release();
    return PFM_OK;
}

int pfm_vad_detector_push(pfm_vad_detector* d, const double* decibel, int n_db, const float* p_sil, int n,
                          int is_final, int streaming, int32_t* segs, int cap, int32_t* n_segs) {
    if (!d || (n_db > 0 && !decibel) || (n > 0 && !p_sil) || !n_segs || (cap > 0 && !segs))
        return pfm_fail(PFM_E_ARG, "pfm_vad_detector_push: null argument");
    if (n_db < 0 || n < 0 || cap < 0) return pfm_fail(PFM_E_ARG, "pfm_vad_detector_push: bad sizes");
    d->db.insert(d->db.end(), decibel, decibel + n_db);
    d->ps.insert(d->ps.end(), p_sil, p_sil + n);
    d->frm_cnt += n;
    if ((int)d->db.size() < d->frm_cnt)
        return pfm_fail(PFM_E_ARG, "pfm_vad_detector_push: fewer decibel frames than posterior frames");
    if (d->state != VS_END) {   // DetectCommonFrames / DetectLastFrames (:755-780)
        for (int i = n - 1; i >= 0; --i) {
            const int t = d->frm_cnt - 1 - i;
            const int st = d->frame_state(t);
            if (st == -100 || d->detect_one(st, t, is_final && i == 0))
                return pfm_fail(PFM_E_STATE, "pfm_vad_detector_push: reset with an open segment");
        }
    }
    // forward() output (:566-613)
    int k = 0;
    const int n_out = (int)d->out.size();
    for (int i = d->out_offset; i < n_out; ++i) {
        const VadSeg& s = d->out[i];
        int beg, end;
        if (streaming) {
            if (!s.has_start) continue;
            if (!d->next_seg && !s.has_end) continue;
            beg = d->next_seg ? s.start_ms : -1;
            if (s.has_end) { end = s.end_ms; d->next_seg = true; d->out_offset += 1; }
            else { end = -1; d->next_seg = false; }
        } else {
            if (!is_final && (!s.has_start || !s.has_end)) continue;
            beg = s.start_ms; end = s.end_ms;
            d->out_offset += 1;
        }
        if (k < cap) { segs[2 * k] = beg; segs[2 * k + 1] = end; }
        ++k;
    }
    *n_segs = k;
    if (k > cap) return pfm_fail(PFM_E_ARG, "pfm_vad_detector_push: segment capacity too small");
    return PFM_OK;
}

void pfm_vad_detector_destroy(pfm_vad_detector* d) { delete d; }

}  // extern "C"
