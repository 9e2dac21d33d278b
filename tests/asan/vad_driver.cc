// Host sanitizer driver for the FSMN-VAD state machine (funasr_amd/csrc/vad_detector.hip), built by
// tests/test_host_sanitize.py with g++ -fsanitize=address,undefined. Reads a chunk schedule from a binary file:
//   int32 n_chunks, int32 streaming; per chunk: int32 n_db, int32 n, float64 db[n_db], float32 p_sil[n], int32 final
// and prints every segment the detector returns as "beg end" lines (streaming: -1 for an open side).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "pfm.h"

static thread_local std::string g_err;
int pfm_fail(int code, const char* msg) { g_err = msg; return code; }

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t nc = 0, streaming = 0;
    if (fread(&nc, 4, 1, f) != 1 || fread(&streaming, 4, 1, f) != 1) return 2;
    pfm_vad_opts o;
    pfm_vad_opts_default(&o);
    pfm_vad_detector* d = nullptr;
    if (pfm_vad_detector_create(&o, &d) != PFM_OK) return 3;
    std::vector<int32_t> segs(2 * 4096);
    for (int c = 0; c < nc; ++c) {
        int32_t ndb = 0, n = 0, fin = 0;
        if (fread(&ndb, 4, 1, f) != 1 || fread(&n, 4, 1, f) != 1) return 2;
        std::vector<double> db(ndb);
        std::vector<float> ps(n);
        if ((ndb && fread(db.data(), 8, ndb, f) != (size_t)ndb) || (n && fread(ps.data(), 4, n, f) != (size_t)n) ||
            fread(&fin, 4, 1, f) != 1)
            return 2;
        int32_t ns = 0;
        const int rc = pfm_vad_detector_push(d, ndb ? db.data() : nullptr, ndb, n ? ps.data() : nullptr, n, fin,
                                             streaming, segs.data(), 4096, &ns);
        if (rc != PFM_OK) { printf("error %d %s\n", rc, g_err.c_str()); break; }
        for (int i = 0; i < ns; ++i) printf("%d %d\n", segs[2 * i], segs[2 * i + 1]);
    }
    pfm_vad_detector_destroy(d);
    fclose(f);
    return 0;
}
