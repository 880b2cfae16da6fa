// ctl_anim.h — per-vertex, per-triangle and per-box arithmetic shared by the
// host scene compiler and the device animation kernels (anim.hip):
//   woop_set_hd        TriIntersectorData::setData    Engine/TriIntersectorData.cu:5-18
//   float_to_half      half(float)                    Math/half.h:21-60 (host branch; equals
//                                                     __float2half_rn, round to nearest even)
//   triangle_set_data  TriangleData::setData          Engine/TriangleData.cu:35-63
//   skin_vertex        g_ComputeVertices / d_Compute  Engine/AnimatedMesh.cu:13-43
//   instance_box       the node world box of ctl_host_scene_compile (8 transformed
//                      corners of the mesh box + 1e-6 relative slack)
#pragma once
#include "ctl_math.h"
#include "../../include/ctl_trace.h"

namespace ctl {

CTL_HD void woop_set_hd(f3 a, f3 b, f3 c, float out[12]) {
    m44 m;
    m.set_col(0, mk4(a - c, 0));
    m.set_col(1, mk4(b - c, 0));
    m.set_col(2, mk4(cross(a - c, b - c), 0));
    m.set_col(3, mk4(c, 1));
    m = inverse(m);
    f4 A = mk4(m.at(2, 0), m.at(2, 1), m.at(2, 2), -m.at(2, 3));
    f4 B = m.row(0), C = m.row(1);
    out[0] = A.x; out[1] = A.y; out[2] = A.z; out[3] = A.w;
    out[4] = B.x; out[5] = B.y; out[6] = B.z; out[7] = B.w;
    out[8] = C.x; out[9] = C.y; out[10] = C.z; out[11] = C.w;
}

CTL_HD uint16_t float_to_half(float f) {
    uint32_t ia = (uint32_t)f_bits(f);
    uint16_t ir = (ia >> 16) & 0x8000;
    if ((ia & 0x7f800000) == 0x7f800000) {
        if ((ia & 0x7fffffff) == 0x7f800000) ir |= 0x7c00;
        else ir = 0x7fff;
    } else if ((ia & 0x7f800000) >= 0x33000000) {
        int shift = (int)((ia >> 23) & 0xff) - 127;
        if (shift > 15) ir |= 0x7c00;
        else {
            ia = (ia & 0x007fffff) | 0x00800000;
            if (shift < -14) { ir |= ia >> (-1 - shift); ia = ia << (32 - (-1 - shift)); }
            else { ir |= ia >> (24 - 11); ia = ia << (32 - (24 - 11)); ir = ir + ((14 + shift) << 10); }
            if ((ia > 0x80000000u) || ((ia == 0x80000000u) && (ir & 1))) ir++;
        }
    }
    return ir;
}

// TriangleData::setData on a record whose material byte and UV halves (w[1]
// high half, w[5..7]) are already set.  The UVs are read back through half's
// float conversion: the host quirk decode when the record is built on the host
// (compile), IEEE (__half2float) when built on the device (animation).
CTL_HD void triangle_set_data(uint32_t w[8], f3 v0, f3 v1, f3 v2, f3 n0, f3 n1, f3 n2, bool uv_host_decode) {
    f2 t0 = mk2(half_to_float(w[5] & 0xffff, uv_host_decode), half_to_float(w[5] >> 16, uv_host_decode));
    f2 t1 = mk2(half_to_float(w[6] & 0xffff, uv_host_decode), half_to_float(w[6] >> 16, uv_host_decode));
    f2 t2 = mk2(half_to_float(w[7] & 0xffff, uv_host_decode), half_to_float(w[7] >> 16, uv_host_decode));
    f3 dP1 = v1 - v0, dP2 = v2 - v0;
    f2 dUV1 = t1 - t0, dUV2 = t2 - t0;
    float determinant = dUV1.x * dUV2.y - dUV1.y * dUV2.x;
    f3 dpdu, dpdv;
    if (determinant == 0) {
        f3 a, b, n = normalize(cross(dP1, dP2));
        coordinate_system(n, a, b);
        dpdu = a; dpdv = b;
    } else {
        float invDet = 1.0f / determinant;
        dpdu = ((dUV2.y * dP1 - dUV1.y * dP2) * invDet);
        dpdv = ((-dUV2.x * dP1 + dUV1.x * dP2) * invDet);
    }
    w[0] = (uint32_t)normal_encode16(n0) | ((uint32_t)normal_encode16(n1) << 16);
    w[1] = (uint32_t)normal_encode16(n2) | (w[1] & 0xffff0000u);
    w[2] = float_to_half(dpdu.x) | ((uint32_t)float_to_half(dpdu.y) << 16);
    w[3] = float_to_half(dpdu.z) | ((uint32_t)float_to_half(dpdv.x) << 16);
    w[4] = float_to_half(dpdv.y) | ((uint32_t)float_to_half(dpdv.z) << 16);
}

// d_Compute (AnimatedMesh.cu:13-27): sum over the 8 (bone, weight/255) slots;
// w[i] = (weight byte i) / 255.0f, the same for both frames.  Bone j's matrix
// starts at bones + stride * j (the device pads the stride against LDS bank
// conflicts).
CTL_HD m44 skin_matrix(const float* bones, uint32_t stride, uint64_t idx, const float w[8]) {
    m44 mat;
    for (int k = 0; k < 16; k++) mat.d[k] = 0.0f;
    for (int i = 0; i < 8; i++) {
        const uint32_t j = (uint32_t)(idx & 0xff);
        idx >>= 8;
        const float* m = bones + stride * j;
        for (int k = 0; k < 16; k++) mat.d[k] = mat.d[k] + m[k] * w[i];
    }
    return mat;
}

// g_ComputeVertices (AnimatedMesh.cu:29-43): position and normal between two frames.
CTL_HD void skin_vertex(const ctl_anim_vertex& v, const float* bones0, const float* bones1, uint32_t stride, float t,
                        f3& P, f3& N) {
    float w[8];
    uint64_t wgt = v.bone_weights;
    for (int i = 0; i < 8; i++, wgt >>= 8) w[i] = (float)(uint32_t)(wgt & 0xff) / 255.0f;
    const m44 m0 = skin_matrix(bones0, stride, v.bone_indices, w);
    const m44 m1 = skin_matrix(bones1, stride, v.bone_indices, w);
    const f3 p = mk3(v.pos[0], v.pos[1], v.pos[2]), n = mk3(v.normal[0], v.normal[1], v.normal[2]);
    const f3 p0 = xform_point(m0, p), p1 = xform_point(m1, p);
    P = p0 * (1.0f - t) + p1 * t;   // math::lerp (MathFunc.h:161)
    const f3 n0 = xform_dir(m0, n), n1 = xform_dir(m1, n);
    N = normalize(n0 * (1.0f - t) + n1 * t);
}

CTL_HD void instance_box(const m44& xf, const float lo[3], const float hi[3], float olo[3], float ohi[3]) {
    for (int k = 0; k < 3; k++) { olo[k] = 3.402823466e+38f; ohi[k] = -3.402823466e+38f; }
    for (int c = 0; c < 8; c++) {
        f3 p = mk3((c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]);
        f3 q = xform_point(xf, p);
        float qq[3] = {q.x, q.y, q.z};
        for (int k = 0; k < 3; k++) { olo[k] = tmin(olo[k], qq[k]); ohi[k] = tmax(ohi[k], qq[k]); }
    }
    // conservative slack against rounding of the corner transform
    for (int k = 0; k < 3; k++) {
        float ext = tmax(fabsf(olo[k]), fabsf(ohi[k])) * 1e-6f + 1e-30f;
        olo[k] -= ext; ohi[k] += ext;
    }
}

}  // namespace ctl
