/*
 * fused_ssim.h -- C ABI of the fused SSIM map (libgsr_hip.so, csrc/ssim.hip): the drop-in
 * behind the reference's optional `fused_ssim` module (submodule fused-ssim, un-vendored;
 * used by train.py:31-35,121-124) and the `fusedssim` / `fusedssim_backward` ops that
 * utils/loss_utils.py:17-38 imports from diff_gaussian_rasterization._C.
 *
 * Semantics: the reference's PyTorch SSIM (utils/loss_utils.py:56-86) -- 11x11 Gaussian window
 * (sigma 1.5), zero ("same") padding, per plane.  Images are float32 [planes, H, W] device
 * arrays (planes = batch x channels).  Same conventions as gsr.h: explicit stream, int status
 * + gsr_last_error(), nothing throws.
 */
#ifndef FUSED_SSIM_H_INCLUDED
#define FUSED_SSIM_H_INCLUDED

#ifdef __cplusplus
extern "C" {
#endif

/* ssim_map = SSIM(img1, img2) per pixel.  With dm_dmu1 / dm_dsigma1_sq / dm_dsigma12 all
 * non-NULL (training), also writes the map's partial derivatives the backward needs:
 * d map / d mu1 (including mu1's share in sigma1_sq and sigma12), d map / d sigma1_sq and
 * d map / d sigma12. */
int gsr_ssim_forward(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                     float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, void* stream);

/* dL_dimg1 from dL_dmap and the forward's partial derivatives. */
int gsr_ssim_backward(int planes, int H, int W, float C1, float C2, const float* img1, const float* img2,
                      const float* dL_dmap, const float* dm_dmu1, const float* dm_dsigma1_sq,
                      const float* dm_dsigma12, float* dL_dimg1, void* stream);

#ifdef __cplusplus
}
#endif

#endif
