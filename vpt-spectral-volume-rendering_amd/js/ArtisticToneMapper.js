'use strict';
// ArtisticToneMapper — drop-in for the reference's WebGPUArtisticToneMapper
// (src/js/tonemappers/WebGPUArtisticToneMapper.js, base WebGPUAbstractToneMapper.js,
// shader src/wgsl/tonemappers/ArtisticToneMapper.wgsl:38-48): the rgba16float
// radiance image of a MCMSpectralComputeRenderer -> rgba8unorm, on the GPU
// (HIP kernel k_tonemap_artistic through the C-ABI vptmcm_tonemap_artistic).
//
// Same properties (low, high, mid, saturation, gamma; js:12-48) and methods
// (render, setTexture, getTexture, setResolution, destroy). The reference passes
// a GPUTexture + sampler; here the "texture" is the renderer whose render target
// the mapper reads (WebGPURenderingContext.js:156-157 passes
// renderer.getTexture(), renderer.getTextureSampler()), and getTexture()
// returns the rgba8 image as a host Uint8Array (R*R*4).
const { PropertyBag } = require('./PropertyBag');
const { native } = require('./MCMSpectralComputeRenderer');

class ArtisticToneMapper extends PropertyBag {
  constructor(device, texture, textureSampler, options = {}) {
    super();
    this._device = device;
    this._resolution = options.resolution !== undefined ? options.resolution : 512;
    this.registerProperties([  // WebGPUArtisticToneMapper.js:12-48
      { name: 'low', label: 'Low', type: 'spinner', value: 0 },
      { name: 'high', label: 'High', type: 'spinner', value: 1 },
      { name: 'mid', label: 'Midtones', type: 'slider', value: 0.5, min: 0.00001, max: 0.99999 },
      { name: 'saturation', label: 'Saturation', type: 'spinner', value: 1 },
      { name: 'gamma', label: 'Gamma', type: 'spinner', value: 2.2, min: 0 },
    ]);
    this.setTexture(texture, textureSampler);
  }

  setTexture(texture, textureSampler) {  // WebGPUAbstractToneMapper.js:26-29
    if (texture && !texture._h) {
      throw new Error('ArtisticToneMapper: the texture source must be a HIP renderer ' +
        '(MCMSpectralComputeRenderer); a host image cannot be tone-mapped on the device');
    }
    this._source = texture || null;
    this._textureSampler = textureSampler;
  }

  setResolution(resolution) {  // WebGPUAbstractToneMapper.js:46-51
    this._resolution = resolution;
    this._image = null;
  }

  render() {  // WebGPUArtisticToneMapper._renderFrame, js:77-122
    if (!this._source) throw new Error('ArtisticToneMapper: no texture set');
    const R = this._source._resolution;
    if (!this._image || this._image.length !== R * R * 4) this._image = new Uint8Array(R * R * 4);
    const params = new Float32Array([this.low, this.mid, this.high, this.saturation, this.gamma]);
    native().tonemapArtistic(this._source._h, params, this._image, R);
  }

  getTexture() {  // the rgba8unorm render buffer (host copy)
    return this._image || null;
  }

  getTextureSampler() {  // clamp-to-edge, linear (WebGPUAbstractToneMapper.js:64-69)
    return { addressModeU: 'clamp-to-edge', addressModeV: 'clamp-to-edge', magFilter: 'linear',
      minFilter: 'linear' };
  }

  destroy() {
    this._image = null;
    this._source = null;
  }
}

// Name -> tone mapper class (WebGPUToneMapperFactory.js); only 'artistic' is GPU-backed here.
function ToneMapperFactory(which) {
  switch (which) {
    case 'artistic': return ArtisticToneMapper;
    default: throw new Error('No suitable class');
  }
}

module.exports = { ArtisticToneMapper, ToneMapperFactory };
