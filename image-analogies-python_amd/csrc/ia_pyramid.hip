// ia_pyramid.hip — GPU preprocessing: the Gaussian pyramid of img_setup
// (image_analogies.py:70-80 -> img_preprocess.py:47-63 -> skimage 0.18.3 pyramid_gaussian) and the
// RGB <-> YIQ matrices (img_preprocess.py:6-22), bit-identical to the package's host restatement
// (ia_amd.img_preprocess, numpy + scipy.ndimage), which is itself within 1e-12 of skimage.
//
// One pyramid_reduce step = scipy.ndimage.gaussian_filter(sigma = 2/3, mode 'reflect', truncate 4:
// 7 taps; axis 0, then axis 1; a colour axis is not smoothed) + skimage resize(order 1,
// anti_aliasing off, clip) to ceil(h/2) x ceil(w/2).  The arithmetic follows the host code
// operation by operation (fp64, no contraction: -ffp-contract=off):
//   correlate1d (scipy ni_filters.c NI_Correlate1D, symmetric kernel):
//     out = x[i] * w[3];  out += (x[i-3] + x[i+3]) * w[0];  ... (x[i-1] + x[i+1]) * w[2]
//   with 'reflect' = half-sample symmetric extension (d c b a | a b c d | d c b a);
//   bilinear: r = (h / oh) * (o + 0.5) - 0.5, r0 = floor, r1 = ceil, dr = r - r0, top =
//     (1 - dc) * tl + dc * tr, bottom = (1 - dc) * bl + dc * br, v = (1 - dr) * top + dr * bottom,
//   clipped to [min, max] of the smoothed image.
// Memory-bound streaming kernels (each level is read and written a few times: HBM roofline);
// intermediate levels stay in HBM, one C call per image.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "ia_internal.h"
#include "ia_launch.h"

#define PY_WG 256

__device__ __forceinline__ int py_reflect(int i, int n) { return ia_reflect(i, n); }

// axis 0 (AXIS = 0: along rows, stride w*ch) or axis 1 (AXIS = 1: along columns, stride ch)
template <int AXIS>
__global__ void __launch_bounds__(PY_WG) k_gauss1d(const double *__restrict__ in, double *__restrict__ out, int h, int w,
                                                    int ch, double w0, double w1, double w2, double w3) {
  const int64_t n = (int64_t)h * w * ch;
  for (int64_t i = (int64_t)blockIdx.x * PY_WG + threadIdx.x; i < n; i += (int64_t)gridDim.x * PY_WG) {
    const int c = (int)(i % ch);
    const int64_t p = i / ch;
    const int x = (int)(p % w), y = (int)(p / w);
    const int L = AXIS == 0 ? h : w, pos = AXIS == 0 ? y : x;
    auto at = [&](int k) {
      const int q = py_reflect(pos + k, L);
      return AXIS == 0 ? in[((int64_t)q * w + x) * ch + c] : in[((int64_t)y * w + q) * ch + c];
    };
    double v = at(0) * w3;
    v += (at(-3) + at(3)) * w0;
    v += (at(-2) + at(2)) * w1;
    v += (at(-1) + at(1)) * w2;
    out[i] = v;
  }
}

// global min / max of the smoothed level (np.clip bounds), two doubles per workgroup, then one
// workgroup folds them (exact: min / max are order-free)
__global__ void __launch_bounds__(PY_WG) k_minmax(const double *__restrict__ x, int64_t n, double *__restrict__ part) {
  __shared__ double smin[PY_WG], smax[PY_WG];
  double lo = DBL_MAX, hi = -DBL_MAX;
  for (int64_t i = (int64_t)blockIdx.x * PY_WG + threadIdx.x; i < n; i += (int64_t)gridDim.x * PY_WG) {
    lo = fmin(lo, x[i]);
    hi = fmax(hi, x[i]);
  }
  smin[threadIdx.x] = lo;
  smax[threadIdx.x] = hi;
  __syncthreads();
  for (int s = PY_WG / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = smin[0];
    part[2 * blockIdx.x + 1] = smax[0];
  }
}
__global__ void __launch_bounds__(PY_WG) k_minmax_fold(double *__restrict__ part, int n) {
  __shared__ double smin[PY_WG], smax[PY_WG];
  double lo = DBL_MAX, hi = -DBL_MAX;
  for (int i = threadIdx.x; i < n; i += PY_WG) {
    lo = fmin(lo, part[2 * i]);
    hi = fmax(hi, part[2 * i + 1]);
  }
  smin[threadIdx.x] = lo;
  smax[threadIdx.x] = hi;
  __syncthreads();
  for (int s = PY_WG / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[0] = smin[0];
    part[1] = smax[0];
  }
}

__global__ void __launch_bounds__(PY_WG) k_bilinear_half(const double *__restrict__ sm, double *__restrict__ out, int h,
                                                          int w, int ch, int oh, int ow, const double *__restrict__ mm) {
  const int64_t n = (int64_t)oh * ow * ch;
  const double fh = (double)h / (double)oh, fw = (double)w / (double)ow;
  const double lo = mm[0], hi = mm[1];
  for (int64_t i = (int64_t)blockIdx.x * PY_WG + threadIdx.x; i < n; i += (int64_t)gridDim.x * PY_WG) {
    const int c = (int)(i % ch);
    const int64_t p = i / ch;
    const int ox = (int)(p % ow), oy = (int)(p / ow);
    const double rr = fh * ((double)oy + 0.5) - 0.5, cc = fw * ((double)ox + 0.5) - 0.5;
    const double fr = floor(rr), fc = floor(cc);
    const int r0 = (int)fr, c0 = (int)fc, r1 = (int)ceil(rr), c1 = (int)ceil(cc);
    const double dr = rr - fr, dc = cc - fc;
    const double tl = sm[((int64_t)r0 * w + c0) * ch + c], tr = sm[((int64_t)r0 * w + c1) * ch + c];
    const double bl = sm[((int64_t)r1 * w + c0) * ch + c], br = sm[((int64_t)r1 * w + c1) * ch + c];
    const double top = (1.0 - dc) * tl + dc * tr;
    const double bottom = (1.0 - dc) * bl + dc * br;
    const double v = (1.0 - dr) * top + dr * bottom;
    out[i] = fmin(fmax(v, lo), hi);
  }
}

// 3x3 colour matrix per pixel, np.einsum('ij,klj->kli', M, img) order: (m0 x0 + m2 x2) + m1 x1
__global__ void __launch_bounds__(PY_WG) k_color3(const double *__restrict__ in, double *__restrict__ out, int64_t npx,
                                                   const double *__restrict__ M) {
  for (int64_t i = (int64_t)blockIdx.x * PY_WG + threadIdx.x; i < npx * 3; i += (int64_t)gridDim.x * PY_WG) {
    const int64_t p = i / 3;
    const int r = (int)(i - p * 3);
    const double x0 = in[3 * p], x1 = in[3 * p + 1], x2 = in[3 * p + 2];
    out[i] = (M[3 * r] * x0 + M[3 * r + 2] * x2) + M[3 * r + 1] * x1;
  }
}

static inline unsigned py_grid(int64_t n) {
  const int64_t g = (n + PY_WG - 1) / PY_WG;
  return (unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

// one pyramid_reduce of in (h, w, ch) -> out (ceil(h/2), ceil(w/2), ch); tmp, sm: h*w*ch doubles,
// mm: >= 2 * 256 doubles
void ia_launch_pyramid_reduce(const double *in, double *out, double *tmp, double *sm, double *mm, int h, int w, int ch,
                              const double *w7, hipStream_t st) {
  const int64_t n = (int64_t)h * w * ch;
  hipLaunchKernelGGL(k_gauss1d<0>, dim3(py_grid(n)), dim3(PY_WG), 0, st, in, tmp, h, w, ch, w7[0], w7[1], w7[2], w7[3]);
  hipLaunchKernelGGL(k_gauss1d<1>, dim3(py_grid(n)), dim3(PY_WG), 0, st, tmp, sm, h, w, ch, w7[0], w7[1], w7[2], w7[3]);
  const unsigned nb = py_grid(n) < 256 ? py_grid(n) : 256;
  hipLaunchKernelGGL(k_minmax, dim3(nb), dim3(PY_WG), 0, st, sm, n, mm);
  hipLaunchKernelGGL(k_minmax_fold, dim3(1), dim3(PY_WG), 0, st, mm, (int)nb);
  const int oh = (h + 1) / 2, ow = (w + 1) / 2;
  hipLaunchKernelGGL(k_bilinear_half, dim3(py_grid((int64_t)oh * ow * ch)), dim3(PY_WG), 0, st, sm, out, h, w, ch, oh, ow,
                     (const double *)mm);
}

void ia_launch_color3(const double *in, double *out, int64_t npx, const double *M, hipStream_t st) {
  hipLaunchKernelGGL(k_color3, dim3(py_grid(npx * 3)), dim3(PY_WG), 0, st, in, out, npx, M);
}
