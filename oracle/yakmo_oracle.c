/*
 * ORACLE (test infrastructure only) -- yakmo k-means++ seeding + seeding-mean
 * centroids.  See yakmo_oracle.h for the disassembly anchors.
 */
#include "yakmo_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int ora_yakmo_seed_means(int N, int D, const float *X, int K, float *centroids, int *labels) {
    if (K >= N || K <= 0 || N <= 0) return -1;
    float *norm = (float *)malloc(sizeof(float) * (size_t)N);
    for (int n = 0; n < N; n++) {
        float s = 0.0f;
        for (int j = 0; j < D; j++) s = s + X[(size_t)n * D + j] * X[(size_t)n * D + j];
        norm[n] = s;
    }
    float *d0 = (float *)calloc((size_t)N, sizeof(float));
    float *d1 = (float *)calloc((size_t)N, sizeof(float));
    int *id = (int *)calloc((size_t)N, sizeof(int));
    float *cum = (float *)calloc((size_t)N, sizeof(float));
    unsigned char *chosen = (unsigned char *)calloc((size_t)N, 1);
    float *cval = (float *)malloc(sizeof(float) * (size_t)D);
    float *sum = (float *)calloc((size_t)K * D, sizeof(float));
    uint32_t *count = (uint32_t *)calloc((size_t)K, sizeof(uint32_t));

    uint64_t x = 123456789ull, y = 362436069ull, z = 521288629ull, w = 88675123ull;
    float total = 0.0f;
    for (int i = 0; i < K; i++) {
        uint64_t t = x ^ (x << 11);
        x = y;
        y = z;
        z = w;
        w = w ^ (w >> 19) ^ t ^ (t >> 8);
        float r = (float)((double)w * 5.42101086242752217e-20 /* 2^-64 */);
        uint32_t idx;
        if (i == 0) {
            float f = floorf(r * (float)N);
            idx = (uint32_t)(int64_t)f;
        } else {
            float target = r * total;
            /* MSVC std::lower_bound over cum[0..N) */
            int64_t first = 0, count_ = N;
            while (count_ > 0) {
                int64_t half = count_ >> 1;
                int64_t mid = first + half;
                if (target > cum[mid]) {
                    first = mid + 1;
                    count_ -= half + 1;
                } else {
                    count_ = half;
                }
            }
            idx = (uint32_t)(int64_t)(float)first;
        }
        while ((uint64_t)idx < (uint64_t)N && chosen[idx]) idx = ((uint64_t)idx < (uint64_t)(N - 1)) ? idx + 1 : 0;
        if ((uint64_t)idx >= (uint64_t)N) idx = (uint32_t)(N - 1);
        chosen[idx] = 1;
        memcpy(cval, X + (size_t)idx * D, sizeof(float) * (size_t)D);
        float cnorm = norm[idx];

        total = 0.0f;
        for (int n = 0; n < N; n++) {
            const float *xp = X + (size_t)n * D;
            float d = (cnorm + norm[n]) + 0.0f;
            for (int j = 0; j < D; j++) d = d - (xp[j] + xp[j]) * cval[j];
            if (i == 0 || d0[n] > d) {
                d1[n] = d0[n];
                d0[n] = d;
                id[n] = i;
            } else if (i == 1) {
                d1[n] = d;
            } else if (d1[n] > d) {
                d1[n] = d;
            }
            if (i < K - 1) {
                total = total + d0[n];
                cum[n] = total;
            } else {
                float *s = sum + (size_t)id[n] * D;
                for (int j = 0; j < D; j++) s[j] = s[j] + xp[j];
                count[id[n]]++;
            }
        }
    }
    for (int c = 0; c < K; c++) {
        float fc = (float)(int64_t)count[c];
        for (int j = 0; j < D; j++) centroids[(size_t)c * D + j] = sum[(size_t)c * D + j] / fc;
    }
    if (labels)
        for (int n = 0; n < N; n++) labels[n] = id[n];
    free(norm);
    free(d0);
    free(d1);
    free(id);
    free(cum);
    free(chosen);
    free(cval);
    free(sum);
    free(count);
    return 0;
}
