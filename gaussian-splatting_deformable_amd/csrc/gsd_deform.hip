// gsd_deform.hip -- fused per-Gaussian SE(3) deform (forward + backward).
//
// Reference: scene/rigid_body.py exp_so3 (:61-65) / exp_se3 (:86-93) with the
// twist normalisation of DirectTemporalNeRF_se3.forward
// (scene/gaussian_model.py:161-165), applied to the means as in
// gaussian_renderer/__init__.py:90-95 (x' = from_homogenous(T [x;1])).  With
// theta = |w| and W = skew(w) (raw w), the reference's
//   R = I + sin(t) W^ + (1-cos t) W^^2,  p = (t I + (1-cos t) W^ + (t - sin t) W^^2) v/t
// equals  R = I + A W + B W^2,  p = v + B W v + C W^2 v  with
//   A = sin t / t,  B = (1 - cos t)/t^2,  C = (t - sin t)/t^3,
// which we evaluate by series below t = 1e-2 (double precision scalars), so
// a zero twist is the identity instead of the reference's 0/0 NaN.
// Rotations (not deformed upstream -- SURVEY.md a2): q' = normalize(q_R (x) q),
// q_R = (cos t/2, sin(t/2)/t * w), Hamilton product as helpers.py:63-70.
// HBM-bound: 52 B read + 28 B written per Gaussian forward.
#include "gsd_kernels.h"

namespace gsd {

struct Se3Coef {
    float A, B, C;        // sin/t, (1-cos)/t^2, (t-sin)/t^3
    float dA, dB, dC;     // A'(t)/t, B'(t)/t, C'(t)/t
    float ch, Sh, dSh;    // cos(t/2), sin(t/2)/t, Sh'(t)/t
};

__device__ __forceinline__ Se3Coef se3_coef(float theta2f) {
    const double t2 = (double)theta2f;
    const double t = sqrt(t2);
    Se3Coef c;
    if (t < 1e-2) {
        const double t4 = t2 * t2, t6 = t4 * t2;
        c.A = (float)(1.0 - t2 / 6.0 + t4 / 120.0 - t6 / 5040.0);
        c.B = (float)(0.5 - t2 / 24.0 + t4 / 720.0 - t6 / 40320.0);
        c.C = (float)(1.0 / 6.0 - t2 / 120.0 + t4 / 5040.0 - t6 / 362880.0);
        c.dA = (float)(-1.0 / 3.0 + t2 / 30.0 - t4 / 840.0);
        c.dB = (float)(-1.0 / 12.0 + t2 / 180.0 - t4 / 6720.0);
        c.dC = (float)(-1.0 / 60.0 + t2 / 1260.0 - t4 / 60480.0);
        c.Sh = (float)(0.5 - t2 / 48.0 + t4 / 3840.0);
        c.dSh = (float)(-1.0 / 24.0 + t2 / 960.0 - t4 / 107520.0);
        c.ch = (float)(1.0 - t2 / 8.0 + t4 / 384.0);
    } else {
        const double s = sin(t), co = cos(t), h = 0.5 * t;
        c.A = (float)(s / t);
        c.B = (float)((1.0 - co) / t2);
        c.C = (float)((t - s) / (t2 * t));
        c.dA = (float)((t * co - s) / (t2 * t));
        c.dB = (float)((t * s - 2.0 * (1.0 - co)) / (t2 * t2));
        c.dC = (float)((3.0 * s - t * co - 2.0 * t) / (t2 * t2 * t));
        c.Sh = (float)(sin(h) / t);
        c.dSh = (float)((0.5 * cos(h) * t - sin(h)) / (t2 * t));
        c.ch = (float)cos(h);
    }
    return c;
}

__device__ __forceinline__ float3 cross3(const float3 a, const float3 b) {
    return make_float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float3 axpy3(float a, const float3 x, const float3 y) {
    return make_float3(a * x.x + y.x, a * x.y + y.y, a * x.z + y.z);
}
__device__ __forceinline__ float3 ld3(const float* p, int i) { return make_float3(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }
__device__ __forceinline__ void st3(float* p, int i, float3 v) {
    p[3 * i] = v.x;
    p[3 * i + 1] = v.y;
    p[3 * i + 2] = v.z;
}

__global__ __launch_bounds__(256) void k_se3_fwd(int P, const float* __restrict__ twist, const float* __restrict__ xin,
                                                 const float* __restrict__ qin, float* __restrict__ xout,
                                                 float* __restrict__ qout) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const float3 w = make_float3(twist[6 * i], twist[6 * i + 1], twist[6 * i + 2]);
    const float3 v = make_float3(twist[6 * i + 3], twist[6 * i + 4], twist[6 * i + 5]);
    const float3 x = ld3(xin, i);
    const Se3Coef c = se3_coef(dot3(w, w));
    const float3 wx = cross3(w, x), wwx = cross3(w, wx);
    const float3 wv = cross3(w, v), wwv = cross3(w, wv);
    float3 o = make_float3(x.x + v.x, x.y + v.y, x.z + v.z);
    o = axpy3(c.A, wx, o);
    o = axpy3(c.B, make_float3(wwx.x + wv.x, wwx.y + wv.y, wwx.z + wv.z), o);
    o = axpy3(c.C, wwv, o);
    st3(xout, i, o);
    if (qin) {
        const float4 q = reinterpret_cast<const float4*>(qin)[i];
        const float3 qv = make_float3(q.y, q.z, q.w);
        const float3 wq = cross3(w, qv);
        float4 r;
        r.x = c.ch * q.x - c.Sh * dot3(w, qv);
        r.y = c.ch * qv.x + c.Sh * (q.x * w.x + wq.x);
        r.z = c.ch * qv.y + c.Sh * (q.x * w.y + wq.y);
        r.w = c.ch * qv.z + c.Sh * (q.x * w.z + wq.z);
        const float n = fmaxf(sqrtf(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w), 1e-12f);  // F.normalize
        reinterpret_cast<float4*>(qout)[i] = make_float4(r.x / n, r.y / n, r.z / n, r.w / n);
    }
}

__global__ __launch_bounds__(256) void k_se3_bwd(int P, const float* __restrict__ twist, const float* __restrict__ xin,
                                                 const float* __restrict__ qin, const float* __restrict__ gxo,
                                                 const float* __restrict__ gqo, float* __restrict__ gtw,
                                                 float* __restrict__ gxi, float* __restrict__ gqi) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const float3 w = make_float3(twist[6 * i], twist[6 * i + 1], twist[6 * i + 2]);
    const float3 v = make_float3(twist[6 * i + 3], twist[6 * i + 4], twist[6 * i + 5]);
    const float3 x = ld3(xin, i);
    const float3 g = ld3(gxo, i);
    const Se3Coef c = se3_coef(dot3(w, w));
    const float3 wx = cross3(w, x), wwx = cross3(w, wx);
    const float3 wv = cross3(w, v), wwv = cross3(w, wv);
    const float3 wg = cross3(w, g), wwg = cross3(w, wg);
    // dL/dx = R^T g = g - A w x g + B w x (w x g)
    st3(gxi, i, make_float3(g.x - c.A * wg.x + c.B * wwg.x, g.y - c.A * wg.y + c.B * wwg.y,
                            g.z - c.A * wg.z + c.B * wwg.z));
    // dL/dv = (I + B W + C W^2)^T g = g - B w x g + C w x (w x g)
    const float3 gv = make_float3(g.x - c.B * wg.x + c.C * wwg.x, g.y - c.B * wg.y + c.C * wwg.y,
                                  g.z - c.B * wg.z + c.C * wwg.z);
    // dL/dw: scalar-coefficient terms + explicit cross-product terms
    const float gu1 = dot3(g, wx);
    const float gu2 = dot3(g, wwx) + dot3(g, wv);
    const float gu3 = dot3(g, wwv);
    const float s = c.dA * gu1 + c.dB * gu2 + c.dC * gu3;
    const float wxd = dot3(w, x), wvd = dot3(w, v), wgd = dot3(w, g), xg = dot3(x, g), vg = dot3(v, g);
    const float3 xcg = cross3(x, g), vcg = cross3(v, g);
    float3 gw;
    gw.x = s * w.x + c.A * xcg.x + c.B * (wxd * g.x + x.x * wgd - 2.f * w.x * xg + vcg.x) +
           c.C * (wvd * g.x + v.x * wgd - 2.f * w.x * vg);
    gw.y = s * w.y + c.A * xcg.y + c.B * (wxd * g.y + x.y * wgd - 2.f * w.y * xg + vcg.y) +
           c.C * (wvd * g.y + v.y * wgd - 2.f * w.y * vg);
    gw.z = s * w.z + c.A * xcg.z + c.B * (wxd * g.z + x.z * wgd - 2.f * w.z * xg + vcg.z) +
           c.C * (wvd * g.z + v.z * wgd - 2.f * w.z * vg);
    if (qin) {
        const float4 q = reinterpret_cast<const float4*>(qin)[i];
        const float3 qv = make_float3(q.y, q.z, q.w);
        const float3 wq = cross3(w, qv);
        const float wqd = dot3(w, qv);
        float4 r;
        r.x = c.ch * q.x - c.Sh * wqd;
        r.y = c.ch * qv.x + c.Sh * (q.x * w.x + wq.x);
        r.z = c.ch * qv.y + c.Sh * (q.x * w.y + wq.y);
        r.w = c.ch * qv.z + c.Sh * (q.x * w.z + wq.z);
        const float nraw = sqrtf(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
        const float4 go = reinterpret_cast<const float4*>(gqo)[i];
        float4 gr;  // through F.normalize(x) = x / max(|x|, eps)
        if (nraw > 1e-12f) {
            const float inv = 1.f / nraw;
            const float4 u = make_float4(r.x * inv, r.y * inv, r.z * inv, r.w * inv);
            const float ug = u.x * go.x + u.y * go.y + u.z * go.z + u.w * go.w;
            gr = make_float4((go.x - u.x * ug) * inv, (go.y - u.y * ug) * inv, (go.z - u.z * ug) * inv,
                             (go.w - u.w * ug) * inv);
        } else {
            const float inv = 1e12f;
            gr = make_float4(go.x * inv, go.y * inv, go.z * inv, go.w * inv);
        }
        const float gw0 = gr.x;
        const float3 gvq = make_float3(gr.y, gr.z, gr.w);
        // dL/dq
        const float3 gxw = cross3(gvq, w);
        float4 gq;
        gq.x = c.ch * gw0 + c.Sh * dot3(w, gvq);
        gq.y = -c.Sh * gw0 * w.x + c.ch * gvq.x + c.Sh * gxw.x;
        gq.z = -c.Sh * gw0 * w.y + c.ch * gvq.y + c.Sh * gxw.y;
        gq.w = -c.Sh * gw0 * w.z + c.ch * gvq.z + c.Sh * gxw.z;
        reinterpret_cast<float4*>(gqi)[i] = gq;
        // dL/dw through q_R
        const float qg = dot3(qv, gvq);
        const float3 rwq = make_float3(q.x * w.x + wq.x, q.x * w.y + wq.y, q.x * w.z + wq.z);
        const float rg = dot3(rwq, gvq);
        const float3 qcg = cross3(qv, gvq);
        const float sw = gw0 * (-0.5f * c.Sh * q.x - wqd * c.dSh) - 0.5f * c.Sh * qg + c.dSh * rg;
        gw.x += sw * w.x - gw0 * c.Sh * qv.x + c.Sh * (q.x * gvq.x + qcg.x);
        gw.y += sw * w.y - gw0 * c.Sh * qv.y + c.Sh * (q.x * gvq.y + qcg.y);
        gw.z += sw * w.z - gw0 * c.Sh * qv.z + c.Sh * (q.x * gvq.z + qcg.z);
    }
    gtw[6 * i] = gw.x;
    gtw[6 * i + 1] = gw.y;
    gtw[6 * i + 2] = gw.z;
    gtw[6 * i + 3] = gv.x;
    gtw[6 * i + 4] = gv.y;
    gtw[6 * i + 5] = gv.z;
}

void launch_se3_fwd(int P, const float* twist, const float* xin, const float* qin, float* xout, float* qout,
                    hipStream_t s) {
    if (P > 0) hipLaunchKernelGGL(k_se3_fwd, dim3((P + 255) / 256), dim3(256), 0, s, P, twist, xin, qin, xout, qout);
}
void launch_se3_bwd(int P, const float* twist, const float* xin, const float* qin, const float* gxo, const float* gqo,
                    float* gtw, float* gxi, float* gqi, hipStream_t s) {
    if (P > 0)
        hipLaunchKernelGGL(k_se3_bwd, dim3((P + 255) / 256), dim3(256), 0, s, P, twist, xin, qin, gxo, gqo, gtw, gxi,
                           gqi);
}

}  // namespace gsd
