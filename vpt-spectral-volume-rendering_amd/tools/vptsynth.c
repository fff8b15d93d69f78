/*
 * vptsynth.c — synthetic benchmark inputs (BASELINE.md "Synthetic configs").
 *
 * The reference ships no benchmark volumes; its only generator is
 * py_notebooks/generate_test_volume.ipynb (sphere-in-cube / two spheres,
 * reproduced in numpy by vptmcm/configs.py). Configs C2/C3/C5 need large
 * procedural volumes, defined here:
 *
 *   fBm of Perlin gradient noise with a PCG-hashed lattice
 *     voxel (i,j,k) samples p = ((i+.5)/W, (j+.5)/H, (k+.5)/D)
 *     n(p) = sum_{o<octaves} 0.5^o * noise(p * f0 * 2^o, seed + o) / sum 0.5^o
 *     u8   = clamp(floor(255 * (0.5 + 0.5 n) + 0.5), 0, 255)
 *   noise: 12 cube-edge gradients chosen by the lattice hash
 *     h = pcg(pcg(pcg(pcg(seed) + ix) + iy) + iz), quintic fade.
 * All arithmetic is IEEE double, so the volume is identical on every host.
 * Output layout is x-fastest (writeTexture order).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

static inline uint32_t pcg(uint32_t v) {
    uint32_t x = v * 747796405u + 2891336453u;
    x = ((x >> ((x >> 28u) + 4u)) ^ x) * 277803737u;
    return (x >> 22u) ^ x;
}

static const double G[12][3] = {{1, 1, 0},  {-1, 1, 0},  {1, -1, 0}, {-1, -1, 0},
                                 {1, 0, 1},  {-1, 0, 1},  {1, 0, -1}, {-1, 0, -1},
                                 {0, 1, 1},  {0, -1, 1},  {0, 1, -1}, {0, -1, -1}};

static inline double fade(double t) { return t * t * t * (t * (t * 6.0 - 15.0) + 10.0); }
static inline double lerpd(double a, double b, double t) { return a + t * (b - a); }

static double grad_dot(uint32_t seedh, int32_t ix, int32_t iy, int32_t iz, double dx, double dy,
                       double dz) {
    uint32_t h = pcg(pcg(pcg(seedh + (uint32_t)ix) + (uint32_t)iy) + (uint32_t)iz) % 12u;
    return G[h][0] * dx + G[h][1] * dy + G[h][2] * dz;
}

static double noise3(double x, double y, double z, uint32_t seed) {
    uint32_t sh = pcg(seed);
    double fx0 = floor(x), fy0 = floor(y), fz0 = floor(z);
    int32_t ix = (int32_t)fx0, iy = (int32_t)fy0, iz = (int32_t)fz0;
    double dx = x - fx0, dy = y - fy0, dz = z - fz0;
    double u = fade(dx), v = fade(dy), w = fade(dz);
    double n000 = grad_dot(sh, ix, iy, iz, dx, dy, dz);
    double n100 = grad_dot(sh, ix + 1, iy, iz, dx - 1, dy, dz);
    double n010 = grad_dot(sh, ix, iy + 1, iz, dx, dy - 1, dz);
    double n110 = grad_dot(sh, ix + 1, iy + 1, iz, dx - 1, dy - 1, dz);
    double n001 = grad_dot(sh, ix, iy, iz + 1, dx, dy, dz - 1);
    double n101 = grad_dot(sh, ix + 1, iy, iz + 1, dx - 1, dy, dz - 1);
    double n011 = grad_dot(sh, ix, iy + 1, iz + 1, dx, dy - 1, dz - 1);
    double n111 = grad_dot(sh, ix + 1, iy + 1, iz + 1, dx - 1, dy - 1, dz - 1);
    double x00 = lerpd(n000, n100, u), x10 = lerpd(n010, n110, u);
    double x01 = lerpd(n001, n101, u), x11 = lerpd(n011, n111, u);
    return lerpd(lerpd(x00, x10, v), lerpd(x01, x11, v), w);
}

typedef struct {
    uint8_t* out;
    uint32_t W, H, D, z0, z1, seed;
    int octaves;
    double f0;
} fbm_job;

static void* fbm_run(void* a) {
    fbm_job* j = (fbm_job*)a;
    double norm = 0.0;
    for (int o = 0; o < j->octaves; o++) norm += ldexp(1.0, -o);
    for (uint32_t k = j->z0; k < j->z1; k++) {
        double pz = (k + 0.5) / j->D;
        for (uint32_t jj = 0; jj < j->H; jj++) {
            double py = (jj + 0.5) / j->H;
            uint8_t* row = j->out + ((size_t)k * j->H + jj) * j->W;
            for (uint32_t i = 0; i < j->W; i++) {
                double px = (i + 0.5) / j->W;
                double n = 0.0;
                for (int o = 0; o < j->octaves; o++) {
                    double f = j->f0 * ldexp(1.0, o);
                    n += ldexp(1.0, -o) * noise3(px * f, py * f, pz * f, j->seed + (uint32_t)o);
                }
                n /= norm;
                double v = floor(255.0 * (0.5 + 0.5 * n) + 0.5);
                row[i] = (uint8_t)(v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v));
            }
        }
    }
    return NULL;
}

/* Fill out[W*H*D] with the fBm volume. */
int vs_fbm(uint8_t* out, uint32_t W, uint32_t H, uint32_t D, uint32_t seed, int octaves,
           double base_freq, int nthreads) {
    if (!out || !W || !H || !D || octaves < 1) return -1;
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > D) nthreads = (int)D;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    fbm_job* jobs = (fbm_job*)malloc(sizeof(fbm_job) * nthreads);
    if (!th || !jobs) { free(th); free(jobs); return -1; }
    for (int t = 0; t < nthreads; t++) {
        fbm_job j = {out, W, H, D, (uint32_t)((uint64_t)D * t / nthreads),
                     (uint32_t)((uint64_t)D * (t + 1) / nthreads), seed, octaves, base_freq};
        jobs[t] = j;
        pthread_create(&th[t], NULL, fbm_run, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* Exposed for the generator's own known-answer test. */
double vs_noise3(double x, double y, double z, uint32_t seed) { return noise3(x, y, z, seed); }
