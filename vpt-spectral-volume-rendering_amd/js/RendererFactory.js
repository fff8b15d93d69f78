'use strict';
// Name -> renderer class (WebGPURendererFactory.js:12-27). Only the spectral
// MCM compute renderer is provided by this package; other names throw the
// reference's error.
const { MCMSpectralComputeRenderer } = require('./MCMSpectralComputeRenderer');

function RendererFactory(which) {
  switch (which) {
    case 'mcm-spectral-compute': return MCMSpectralComputeRenderer;
    default: throw new Error('No suitable class');
  }
}

module.exports = { RendererFactory };
