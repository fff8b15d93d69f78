'use strict';
// Minimal column-major 4x4 matrix helpers for the renderer's camera path.
//
// The reference computes mvpInverse with gl-matrix 3.4.1 (Float32Array storage,
// double-precision intermediates): WebGPUMCMSpectralComputeRenderer.js:266-274,
// Transform.js:64-70, PerspectiveCamera.js:9-17. These helpers follow the same
// textbook formulas with the same evaluation order (2x2 sub-determinants for
// the inverse, row-by-column sums for the product) so the Float32 results are
// bit-identical; tests/js/test_host.js pins them against golden bits produced
// by the reference's own gl-matrix (tests/golden/mvp_inverse.json).

function create() {
  const m = new Float32Array(16);
  m[0] = m[5] = m[10] = m[15] = 1;
  return m;
}

function fromTranslation(out, v) {
  out.fill(0);
  out[0] = out[5] = out[10] = out[15] = 1;
  out[12] = v[0]; out[13] = v[1]; out[14] = v[2];
  return out;
}

// out = a * b
function multiply(out, a, b) {
  const a0 = [a[0], a[1], a[2], a[3]], a1 = [a[4], a[5], a[6], a[7]];
  const a2 = [a[8], a[9], a[10], a[11]], a3 = [a[12], a[13], a[14], a[15]];
  for (let c = 0; c < 4; c++) {
    const x = b[4 * c], y = b[4 * c + 1], z = b[4 * c + 2], w = b[4 * c + 3];
    for (let r = 0; r < 4; r++) {
      out[4 * c + r] = x * a0[r] + y * a1[r] + z * a2[r] + w * a3[r];
    }
  }
  return out;
}

// Laplace expansion by complementary 2x2 minors of the top and bottom row pairs.
function invert(out, m) {
  const m00 = m[0], m01 = m[1], m02 = m[2], m03 = m[3];
  const m10 = m[4], m11 = m[5], m12 = m[6], m13 = m[7];
  const m20 = m[8], m21 = m[9], m22 = m[10], m23 = m[11];
  const m30 = m[12], m31 = m[13], m32 = m[14], m33 = m[15];
  const s0 = m00 * m11 - m01 * m10, s1 = m00 * m12 - m02 * m10, s2 = m00 * m13 - m03 * m10;
  const s3 = m01 * m12 - m02 * m11, s4 = m01 * m13 - m03 * m11, s5 = m02 * m13 - m03 * m12;
  const c0 = m20 * m31 - m21 * m30, c1 = m20 * m32 - m22 * m30, c2 = m20 * m33 - m23 * m30;
  const c3 = m21 * m32 - m22 * m31, c4 = m21 * m33 - m23 * m31, c5 = m22 * m33 - m23 * m32;
  let det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
  if (!det) return null;
  det = 1 / det;
  out[0] = (m11 * c5 - m12 * c4 + m13 * c3) * det;
  out[1] = (m02 * c4 - m01 * c5 - m03 * c3) * det;
  out[2] = (m31 * s5 - m32 * s4 + m33 * s3) * det;
  out[3] = (m22 * s4 - m21 * s5 - m23 * s3) * det;
  out[4] = (m12 * c2 - m10 * c5 - m13 * c1) * det;
  out[5] = (m00 * c5 - m02 * c2 + m03 * c1) * det;
  out[6] = (m32 * s2 - m30 * s5 - m33 * s1) * det;
  out[7] = (m20 * s5 - m22 * s2 + m23 * s1) * det;
  out[8] = (m10 * c4 - m11 * c2 + m13 * c0) * det;
  out[9] = (m01 * c2 - m00 * c4 - m03 * c0) * det;
  out[10] = (m30 * s4 - m31 * s2 + m33 * s0) * det;
  out[11] = (m21 * s2 - m20 * s4 - m23 * s0) * det;
  out[12] = (m11 * c1 - m10 * c3 - m12 * c0) * det;
  out[13] = (m00 * c3 - m01 * c1 + m02 * c0) * det;
  out[14] = (m31 * s1 - m30 * s3 - m32 * s0) * det;
  out[15] = (m20 * s3 - m21 * s1 + m22 * s0) * det;
  return out;
}

// OpenGL-style [-1, 1] depth perspective (gl-matrix's perspective/perspectiveNO).
function perspective(out, fovy, aspect, near, far) {
  const f = 1 / Math.tan(fovy / 2);
  out.fill(0);
  out[0] = f / aspect;
  out[5] = f;
  out[11] = -1;
  if (far !== null && far !== undefined && far !== Infinity) {
    const nf = 1 / (near - far);
    out[10] = (far + near) * nf;
    out[14] = 2 * far * near * nf;
  } else {
    out[10] = -1;
    out[14] = -2 * near;
  }
  return out;
}

// rotation matrix of a unit quaternion [x, y, z, w]
function fromQuat(out, q) {
  const x = q[0], y = q[1], z = q[2], w = q[3];
  const x2 = x + x, y2 = y + y, z2 = z + z;
  const xx = x * x2, yx = y * x2, yy = y * y2, zx = z * x2, zy = z * y2, zz = z * z2;
  const wx = w * x2, wy = w * y2, wz = w * z2;
  out[0] = 1 - yy - zz; out[1] = yx + wz; out[2] = zx - wy; out[3] = 0;
  out[4] = yx - wz; out[5] = 1 - xx - zz; out[6] = zy + wx; out[7] = 0;
  out[8] = zx + wy; out[9] = zy - wx; out[10] = 1 - xx - yy; out[11] = 0;
  out[12] = 0; out[13] = 0; out[14] = 0; out[15] = 1;
  return out;
}

function scale(out, a, v) {
  for (let k = 0; k < 4; k++) {
    out[k] = a[k] * v[0];
    out[4 + k] = a[4 + k] * v[1];
    out[8 + k] = a[8 + k] * v[2];
    out[12 + k] = a[12 + k];
  }
  return out;
}

function translate(out, a, v) {
  const x = v[0], y = v[1], z = v[2];
  if (out !== a) for (let k = 0; k < 12; k++) out[k] = a[k];
  for (let r = 0; r < 4; r++) out[12 + r] = a[r] * x + a[4 + r] * y + a[8 + r] * z + a[12 + r];
  return out;
}

function quatInvert(q) {
  const d = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  const inv = d ? 1 / d : 0;
  return new Float32Array([-q[0] * inv, -q[1] * inv, -q[2] * inv, q[3] * inv]);
}

module.exports = { create, fromTranslation, multiply, invert, perspective, fromQuat, scale, translate,
  quatInvert };
