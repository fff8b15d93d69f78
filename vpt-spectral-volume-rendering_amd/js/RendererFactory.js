'use strict';
// Name -> renderer class (WebGPURendererFactory.js:12-27). The spectral MCM
// compute renderer (the north_star path) and its RGB sibling are provided by
// this package; other names throw the reference's error.
const { MCMSpectralComputeRenderer } = require('./MCMSpectralComputeRenderer');
const { MCMComputeRenderer } = require('./MCMComputeRenderer');

function RendererFactory(which) {
  switch (which) {
    case 'mcm-compute': return MCMComputeRenderer;
    case 'mcm-spectral-compute': return MCMSpectralComputeRenderer;
    default: throw new Error('No suitable class');
  }
}

module.exports = { RendererFactory };
