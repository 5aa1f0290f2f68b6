/* TEST INFRASTRUCTURE (CPU-build sanitizer run of the oracle).
 * Runs ofr_estimate_flow over every registry method on a small synthetic
 * pair, built together with optflow_oracle.c under -fsanitize=address,undefined.
 * The of_params records come from the Python registry (BaseOpticalFlow.
 * to_params), written by tests/test_oracle_asan.py as raw struct bytes:
 *   asan_driver PARAMS.bin H W    (PARAMS.bin = n records of sizeof(of_params))
 * Exit 0 when every method returns OF_OK with finite flow. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "optflow.h"

int ofr_estimate_flow(of_params *P, const double *im1, const double *im2, int H, int W, int C,
                      const double *init_uv, double *out_uv, of_stats *st);

int main(int argc, char **argv) {
  if (argc != 4) { fprintf(stderr, "usage: %s PARAMS.bin H W\n", argv[0]); return 2; }
  const int H = atoi(argv[2]), W = atoi(argv[3]);
  FILE *f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 2; }
  fseek(f, 0, SEEK_END);
  const long nb = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (nb <= 0 || nb % (long)sizeof(of_params)) { fprintf(stderr, "bad params file (%ld B)\n", nb); return 2; }
  const int n = (int)(nb / (long)sizeof(of_params));
  of_params *ps = malloc(nb);
  if (fread(ps, 1, nb, f) != (size_t)nb) return 2;
  fclose(f);
  /* RGB pair in [0, 255]: smooth texture, frame 2 = frame 1 shifted by (0.7, -0.4) */
  const long N = (long)H * W;
  double *im1 = malloc(3 * N * sizeof(double)), *im2 = malloc(3 * N * sizeof(double));
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j)
      for (int c = 0; c < 3; ++c) {
        const double y = i, x = j, y2 = i + 0.4, x2 = j - 0.7;
        im1[(i * W + j) * 3 + c] = 127.5 + 60 * sin(0.31 * x + 0.17 * y + c) + 40 * cos(0.23 * y - 0.11 * x * c);
        im2[(i * W + j) * 3 + c] = 127.5 + 60 * sin(0.31 * x2 + 0.17 * y2 + c) + 40 * cos(0.23 * y2 - 0.11 * x2 * c);
      }
  double *uv = malloc(2 * N * sizeof(double));
  int bad = 0;
  for (int m = 0; m < n; ++m) {
    of_stats st;
    memset(&st, 0, sizeof st);
    const int rc = ofr_estimate_flow(&ps[m], im1, im2, H, W, 3, NULL, uv, &st);
    int finite = 1;
    for (long k = 0; k < 2 * N; ++k) finite &= isfinite(uv[k]) != 0;
    printf("method %d rc %d finite %d\n", m, rc, finite);
    bad |= rc != 0;
  }
  free(ps); free(im1); free(im2); free(uv);
  return bad;
}
