/* Host parse throughput of one IVF stream on one thread (vp9h_stream_decode per frame, a
 * fresh stream per repetition): the term that bounds the FFHWAccel path of 8K GOP chains
 * (profiles/r05k). Build (plain or with -pg for gprof) from the host sources directly:
 *   gcc -O2 -std=gnu11 -Iinclude -Iffmpeg-hybrid_amd/csrc -o /tmp/pb tools/parse_bench.c \
 *       ffmpeg-hybrid_amd/csrc/host/vp9h_{bitstream,ivf,synth,webm}.c -lpthread -lm
 * usage: /tmp/pb stream.ivf [reps] */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "vp9hip.h"
int main(int argc, char **argv)
{
    FILE *f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t *buf = malloc(n); fread(buf, 1, n, f); fclose(f);
    int reps = argc > 2 ? atoi(argv[2]) : 1;
    vp9h_ivf_header h; vp9h_ivf_read_header(buf, n, &h);
    struct timespec t0, t1; clock_gettime(CLOCK_MONOTONIC, &t0);
    int frames = 0;
    for (int r = 0; r < reps; r++) {
        vp9h_stream *s; vp9h_stream_open(&s);
        size_t pos = 32; const uint8_t *d; uint32_t sz; int64_t pts; int tr;
        while (vp9h_ivf_read_frame(buf, n, &pos, &d, &sz, &pts, &tr) == 0) {
            vp9h_frame fr; vp9h_frame_info info; memset(&fr, 0, sizeof(fr));
            if (vp9h_stream_decode(s, d, sz, &fr, &info) < 0) { fprintf(stderr, "decode error\n"); return 1; }
            vp9h_frame_free(&fr); frames++;
        }
        vp9h_stream_close(s);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double dt = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    printf("%d frames %.3f s %.2f fps\n", frames, dt, frames / dt);
    return 0;
}
