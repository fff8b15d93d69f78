'use strict';
// Spectrum representation: CIE colour-matching bin means and the packed
// 64-f32 buffer the kernel reads.
//
// computeSpectralCoefficients restates the reference's
// compute_spectral_coefficients (WebGPUMCMSpectralComputeRenderer.js:379-412):
// a box average of the 1-nm CIE table over each bin [lambda_i, lambda_i+1),
// visiting wavelengths from the first bin boundary upward, advancing at most
// one bin per nanometre, stopping after the last bin. The CIE table is the
// caller's (the host application ships it: src/js/utils/Spectrum.js); the
// tests use the golden copy in tests/golden/cie1931.json.

function computeSpectralCoefficients(bins, cie) {
  const nBins = bins.length - 1;
  const x = new Array(nBins).fill(0), y = new Array(nBins).fill(0), z = new Array(nBins).fill(0);
  const weight = new Array(nBins).fill(0);
  const first = cie.first_wavelength !== undefined ? cie.first_wavelength : cie.first_wavelenght;
  const count = cie.length !== undefined ? cie.length : cie.X.length;
  let bin = 0;
  for (let k = 0; k < count; k++) {
    const lambda = first + k * cie.step;
    if (lambda < bins[0]) continue;
    if (lambda >= bins[bin + 1]) bin++;
    if (bin >= nBins) break;
    weight[bin] += 1;
    x[bin] += cie.X[k];
    y[bin] += cie.Y[k];
    z[bin] += cie.Z[k];
  }
  for (let b = 0; b < nBins; b++) {
    x[b] /= weight[b];
    y[b] /= weight[b];
    z[b] /= weight[b];
  }
  return { x, y, z };
}

// [n_bins, lambda_0..lambda_n, xbar.., ybar.., zbar..] in a 64-float buffer (js:311-312)
function packSpectrumBuffer(bins, coeff) {
  const nBins = bins.length - 1;
  if (nBins > 12) throw new Error('at most 12 spectral bins (MAX_N_BINS)');
  const buf = new Float32Array(64);
  buf.set([nBins, ...bins, ...coeff.x, ...coeff.y, ...coeff.z]);
  return buf;
}

const DEFAULT_BINS = [400, 425, 450, 475, 500, 525, 550, 575, 600, 625, 650, 675, 700]; // js:79

module.exports = { computeSpectralCoefficients, packSpectrumBuffer, DEFAULT_BINS };
