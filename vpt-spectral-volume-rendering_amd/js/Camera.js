'use strict';
// Camera node compatible with what the reference renderer reads from its
// camera (WebGPUMCMSpectralComputeRenderer.js:219-220):
//   camera.transform.inverseGlobalMatrix                      (Transform.js:64-70)
//   camera.getComponent(PerspectiveCamera).projectionMatrix   (PerspectiveCamera.js:9-17)
// Defaults are the reference context's camera (WebGPURenderingContext.js:37-39):
// translation [0, 0, 2], identity rotation, fovy 1 rad, aspect 1, near 0.1, far 100.
const mat4 = require('./mat4');

class Transform {
  constructor(opts = {}) {
    this.localTranslation = Float32Array.from(opts.translation || [0, 0, 0]);
    this.localRotation = Float32Array.from(opts.rotation || [0, 0, 0, 1]);
    this.localScale = Float32Array.from(opts.scale || [1, 1, 1]);
  }

  get inverseGlobalMatrix() {
    const inverseScale = new Float32Array([1 / this.localScale[0], 1 / this.localScale[1],
      1 / this.localScale[2]]);
    const inverseRotation = mat4.quatInvert(this.localRotation);
    const inverseTranslation = new Float32Array([-this.localTranslation[0],
      -this.localTranslation[1], -this.localTranslation[2]]);
    const m = mat4.create();
    mat4.scale(m, m, inverseScale);
    mat4.multiply(m, m, mat4.fromQuat(mat4.create(), inverseRotation));
    mat4.translate(m, m, inverseTranslation);
    return m;
  }
}

class PerspectiveCamera {
  constructor(opts = {}) {
    this.fovy = opts.fovy !== undefined ? opts.fovy : 1;
    this.aspect = opts.aspect !== undefined ? opts.aspect : 1;
    this.near = opts.near !== undefined ? opts.near : 0.1;
    this.far = opts.far !== undefined ? opts.far : 100;
  }

  get projectionMatrix() {
    return mat4.perspective(mat4.create(), this.fovy, this.aspect, this.near, this.far);
  }
}

class Camera {
  constructor(opts = {}) {
    this.transform = new Transform({ translation: opts.translation || [0, 0, 2],
      rotation: opts.rotation, scale: opts.scale });
    this.components = [new PerspectiveCamera(opts)];
  }

  getComponent(type) {
    return this.components.find(c => c instanceof type);
  }
}

// invert(P * V * M) with M = translate(-0.5) — the sequence of js:266-274.
function mvpInverse(camera) {
  const modelMatrix = mat4.fromTranslation(mat4.create(), [-0.5, -0.5, -0.5]);
  const viewMatrix = camera.transform.inverseGlobalMatrix;
  const persp = camera.getComponent ? camera.getComponent(PerspectiveCamera) ||
    camera.components.find(c => c && c.projectionMatrix) : null;
  const projectionMatrix = persp.projectionMatrix;
  const matrix = mat4.create();
  mat4.multiply(matrix, modelMatrix, matrix);
  mat4.multiply(matrix, viewMatrix, matrix);
  mat4.multiply(matrix, projectionMatrix, matrix);
  mat4.invert(matrix, matrix);
  return matrix;
}

module.exports = { Camera, Transform, PerspectiveCamera, mvpInverse };
