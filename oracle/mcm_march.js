'use strict';
// mcm_march.js — TEST INFRASTRUCTURE ONLY: the scalar JavaScript re-execution
// of the spectral MCM march (BASELINE.json north_star's "scalar JS/CPU
// re-execution of the same march"), used as bench.py's primary CPU baseline
// and checked bit for bit against oracle/mcm_oracle.c (tests/test_js_march.py).
// Never loaded by the product (js/, napi/, csrc/).
//
// It restates, with Math.fround after every f32 operation, the same march as
// mcm_oracle.c:
//   src/wgsl/renderers/MCMSpectralComputeRenderer.wgsl  render :107-179,
//     reset :213-231, PhotonSpectral :234-326
//   src/wgsl/mixins/random/hash/pcg.wgsl:3-7, squashlinear.wgsl:7-9,
//   random/distribution/{uniformdivision,exponential,disk,square,sphere}.wgsl,
//   src/wgsl/mixins/{unprojectRand,intersectCube}.wgsl
// under the arithmetic specification of DESIGN.md §2 (explicit fma on the
// listed products, a/b = a * RN(1/b), polynomial log/sin/cos, minNum/maxNum).
//
// f32 arithmetic in f64: +, -, *, / and sqrt of two f32 values computed in
// double and rounded once to f32 are correctly rounded (53 >= 2*24 + 2), so
// fround(a op b) is the f32 operation. fma is not: fma32 below rounds the
// exact a*b + c (a*b is exact in double; TwoSum recovers the addition's
// error) to f32 with the tie decided by that error.

const F = Math.fround;
const cvt = new DataView(new ArrayBuffer(4));
const fbits = (x) => { cvt.setFloat32(0, x); return cvt.getUint32(0); };
const bitsf = (u) => { cvt.setUint32(0, u >>> 0); return cvt.getFloat32(0); };

function fma32(a, b, c) {
  const p = a * b;            // exact: 24 + 24 significand bits
  const s = p + c;
  if (!isFinite(s)) return F(s);
  const bb = s - p;
  const err = (p - (s - bb)) + (c - bb);  // p + c == s + err exactly
  const r = F(s);
  if (err === 0) return r;
  const d = s - r;                         // exact (|d| <= half an f32 spacing)
  if (d === 0) return r;                   // s is an f32: err cannot move it past a midpoint
  const other = r + 2 * d;                 // the f32 neighbour if s is a midpoint
  if (F(other) !== other) return r;        // s is not a midpoint: rounding of s stands
  return (err > 0) === (d > 0) ? F(other) : r;
}

const EPS = F(1e-5);                       // wgsl:6
const TWOPI = F(6.2831854820251465);       // constants.wgsl:4
const INV255 = F(0.003921568859368563);
const rcp = (x) => F(1 / x);

function smin(a, b) { if (a !== a) return b; if (b !== b) return a; return b < a ? b : a; }
function smax(a, b) { if (a !== a) return b; if (b !== b) return a; return b > a ? b : a; }

// log (DESIGN.md §2; mcm_oracle.c orc_log)
function specLog(x) {
  let b = fbits(x);
  if (x !== x || (b >>> 31)) return x === 0 ? -Infinity : NaN;
  if (x === 0) return -Infinity;
  if (b === 0x7f800000) return x;
  let e = 0;
  if (b < 0x00800000) { x = F(x * 33554432); b = fbits(x); e = -25; }
  e += (b >>> 23) - 127;
  let m = bitsf((b & 0x007fffff) | 0x3f800000);
  if (m > F(1.41421353816986083984375)) { m = F(m * 0.5); e += 1; }
  const f = F(m - 1);
  const s = F(f / F(2 + f));          // a true division here (RN(f/(2+f)), DESIGN.md §2)
  const z = F(s * s);
  const P = fma32(z, fma32(z, fma32(z, fma32(z, F(0.1818181872367859), F(0.2222222238779068)),
    F(0.2857142984867096)), F(0.4000000059604645)), F(0.6666666865348816));
  const R = F(z * P);
  const lm = fma32(s, R, F(s + s));
  const ef = F(e);
  return fma32(ef, F(0.693115234375), fma32(ef, F(3.194618329871446e-05), lm));
}

// sin/cos: 3-part Cody-Waite by pi/2, Taylor polynomials (mcm_oracle.c spec_sincos)
const sc = [0, 0];
function specSinCos(x) {
  const kf = Math.floor(fma32(x, F(0.6366197466850281), 0.5));
  const r = fma32(-kf, F(7.549790126404332e-08),
    fma32(-kf, F(0.0004837512969970703), fma32(-kf, 1.5703125, x)));
  const z = F(r * r);
  const ps = fma32(z, fma32(z, fma32(z, fma32(z, F(-2.5052107943679403e-08), F(2.7557318844628753e-06)),
    F(-0.00019841270113829523)), F(0.008333333767950535)), F(-0.1666666716337204));
  const s = fma32(F(r * z), ps, r);
  const pc = fma32(z, fma32(z, fma32(z, F(-2.755731998149713e-07), F(2.4801587642286904e-05)),
    F(-0.0013888889225199819)), F(0.0416666679084301));
  const c = fma32(F(z * z), pc, fma32(-0.5, z, 1));
  switch (kf & 3) {
    case 0: sc[0] = s; sc[1] = c; break;
    case 1: sc[0] = c; sc[1] = -s; break;
    case 2: sc[0] = -s; sc[1] = -c; break;
    default: sc[0] = -c; sc[1] = s; break;
  }
}

function rintEven(a) {  // round half to even of a non-negative double
  const fl = Math.floor(a), d = a - fl;
  if (d > 0.5) return fl + 1;
  if (d < 0.5) return fl;
  return fl % 2 === 0 ? fl : fl + 1;
}
function f2h(f) {  // f32 -> binary16, round to nearest even (mcm_oracle.c orc_f2h)
  const x = fbits(f);
  const sign = (x >>> 16) & 0x8000;
  const ax = x & 0x7fffffff;
  if (ax > 0x7f800000) return sign | 0x7e00;
  if (ax >= 0x477ff000) return sign | 0x7c00;
  if (ax < 0x38800000) return sign | rintEven(bitsf(ax) * 16777216);
  let h = ((((ax >>> 23) - 112) << 10) | ((ax & 0x7fffff) >>> 13)) >>> 0;
  const rem = ax & 0x1fff;
  if (rem > 0x1000 || (rem === 0x1000 && (h & 1))) h++;
  return sign | h;
}

const dot3 = (ax, ay, az, bx, by, bz) => fma32(az, bz, fma32(ay, by, F(ax * bx)));

// ------------------------------------------------------------------- RNG
function pcg(v) {  // pcg.wgsl:3-7
  let x = (Math.imul(v, 747796405) + 2891336453) >>> 0;
  x = Math.imul(((x >>> (((x >>> 28) + 4) & 31)) ^ x) >>> 0, 277803737) >>> 0;
  return ((x >>> 22) ^ x) >>> 0;
}
function hash3(x, y, z) {  // squashlinear.wgsl:7-9
  return pcg((Math.imul(19, x) + Math.imul(47, y) + Math.imul(101, z) + 131) >>> 0);
}

// ------------------------------------------------------------- sampling
const clampc = (u) => (u >= -1 ? (u <= 2 ? u : 2) : -1);
const ax = { i0: 0, i1: 0, f: 0 };
function axis(u, n) {
  const x = fma32(clampc(u), n, -0.5);
  const fl = Math.floor(x);
  ax.f = F(x - fl);
  const i = fl;
  ax.i0 = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
  ax.i1 = i + 1 < 0 ? 0 : (i + 1 > n - 1 ? n - 1 : i + 1);
}
const lerp = (a, b, f) => fma32(f, F(b - a), a);

// One renderer's inputs and photon buffer; all arrays may live in shared memory.
class March {
  constructor(o) {
    Object.assign(this, o);  // R, W, H, D, vol, tf, light, spec, photons (ArrayBuffer), u
    this.pw = new Float32Array(this.photons);   // 36 words per photon (144-B stride)
    this.pu = new Uint32Array(this.photons);
    this.st = 0;
    this.p = new Float64Array(34);               // working photon (f32 values)
    this.pi = new Uint32Array(4);                // bounces, samples, bin
    this.dk = [0, 0];
    this.fd = [0, 0, 0, 0];
    this.td = [0, 0, 0, 0];
    this.smp = [0, 0, 0];
    this.sx = 0;
    this.sy = 0;
  }

  uniform() {  // uniformdivision.wgsl:3-6
    this.st = pcg(this.st);
    return F(F(this.st) / 4294967296);
  }

  nBins() { const v = F(this.spec[0] + 0.5); return v > 0 ? (v >>> 0) : 0; }

  sampleVolume(px, py, pz) {  // wgsl:76, clamp-to-edge linear
    const { W, H, D, vol } = this;
    axis(px, W); const x0 = ax.i0, x1 = ax.i1, fx = ax.f;
    axis(py, H); const y0 = ax.i0, y1 = ax.i1, fy = ax.f;
    axis(pz, D); const z0 = ax.i0, z1 = ax.i1, fz = ax.f;
    const V = (i, j, k) => vol[(k * H + j) * W + i];
    const c00 = lerp(V(x0, y0, z0), V(x1, y0, z0), fx);
    const c10 = lerp(V(x0, y1, z0), V(x1, y1, z0), fx);
    const c01 = lerp(V(x0, y0, z1), V(x1, y0, z1), fx);
    const c11 = lerp(V(x0, y1, z1), V(x1, y1, z1), fx);
    return F(lerp(lerp(c00, c10, fy), lerp(c01, c11, fy), fz) * INV255);
  }

  sampleTf(t, d, out) {  // wgsl:77-79: row = density, column = wavelength
    axis(t, 256); const c0 = ax.i0, c1 = ax.i1, fx = ax.f;
    axis(d, 256); const r0 = ax.i0, r1 = ax.i1, fy = ax.f;
    const tf = this.tf;
    for (let ch = 0; ch < 3; ch++) {
      const a = lerp(tf[(r0 * 256 + c0) * 4 + ch], tf[(r0 * 256 + c1) * 4 + ch], fx);
      const b = lerp(tf[(r1 * 256 + c0) * 4 + ch], tf[(r1 * 256 + c1) * 4 + ch], fx);
      out[ch] = F(lerp(a, b, fy) * INV255);
    }
  }

  sampleLight(dx, dy, dz, wavelength) {  // wgsl:62-73
    const t = F(F(wavelength - 400) * rcp(300));
    axis(t, 256);
    const intensity = F(F(lerp(this.light[ax.i0], this.light[ax.i1], ax.f) * INV255) * 5);
    const l = this.u.lightDir;
    const ll = Math.fround(Math.sqrt(dot3(l[0], l[1], l[2], l[0], l[1], l[2])));
    if (ll < EPS) return intensity;
    const il = rcp(ll);
    const lx = F(l[0] * il), ly = F(l[1] * il), lz = F(l[2] * il);
    return smax(F(dot3(dx, dy, dz, lx, ly, lz) * intensity), 0);
  }

  disk(out) {  // disk.wgsl:3-7
    const radius = F(Math.sqrt(this.uniform()));
    const angle = F(TWOPI * this.uniform());
    specSinCos(angle);
    out[0] = F(radius * sc[1]);
    out[1] = F(radius * sc[0]);
  }

  matVec(m, v0, v1, v2, v3, o) {  // column-major mat4 * vec4
    for (let r = 0; r < 4; r++)
      o[r] = fma32(m[12 + r], v3, fma32(m[8 + r], v2, fma32(m[4 + r], v1, F(m[r] * v0))));
  }

  // PhotonSpectral_reset (wgsl:249-266) with unprojectRand / intersectCube
  reset(sx, sy) {
    const u = this.u, p = this.p, pi = this.pi, dk = this.dk, fd = this.fd, td = this.td;
    this.disk(dk);
    const q0 = this.uniform(), q1 = this.uniform();
    this.matVec(u.mvp, fma32(dk[0], u.blur, sx), fma32(dk[1], u.blur, sy), -1, 1, fd);
    this.matVec(u.mvp, fma32(fma32(q0, 2, -1), u.invRes[0], sx),
      fma32(fma32(q1, 2, -1), u.invRes[1], sy), 1, 1, td);
    let iw = rcp(fd[3]);
    const fx = F(fd[0] * iw), fy = F(fd[1] * iw), fz = F(fd[2] * iw);
    iw = rcp(td[3]);
    const tx = F(td[0] * iw), ty = F(td[1] * iw), tz = F(td[2] * iw);
    const vx = F(tx - fx), vy = F(ty - fy), vz = F(tz - fz);
    const il = rcp(F(Math.sqrt(dot3(vx, vy, vz, vx, vy, vz))));
    const dx = F(vx * il), dy = F(vy * il), dz = F(vz * il);
    p[3] = dx; p[4] = dy; p[5] = dz;
    pi[0] = 0;
    const rx = rcp(dx), ry = rcp(dy), rz = rcp(dz);
    const t1x = smin(F(F(0 - fx) * rx), F(F(1 - fx) * rx));
    const t1y = smin(F(F(0 - fy) * ry), F(F(1 - fy) * ry));
    const t1z = smin(F(F(0 - fz) * rz), F(F(1 - fz) * rz));
    const tn = smax(smax(smax(t1x, t1y), t1z), 0);
    p[0] = fma32(tn, dx, fx); p[1] = fma32(tn, dy, fy); p[2] = fma32(tn, dz, fz);
    const nb = this.nBins(), spec = this.spec;
    const minL = spec[1], maxL = spec[nb + 1];
    const lambda = fma32(this.uniform(), F(maxL - minL), minL);
    p[6] = lambda;  // PhotonSpectral_set_wavelength, wgsl:276-290
    pi[2] = (nb - 1) >>> 0;
    for (let i = 1; i < nb; i++) {
      if (lambda < spec[i + 1]) { pi[2] = i - 1; break; }
    }
  }

  addRadiance(radiance) {  // wgsl:292-302
    const nb = this.nBins(), p = this.p;
    const inv = rcp(F(this.pi[1]));
    for (let i = 0; i < nb && i < 12; i++) {
      const tgt = i === this.pi[2] ? radiance : 0;
      p[7 + i] = fma32(F(tgt - p[7 + i]), inv, p[7 + i]);
    }
  }

  load(k) {
    const w = this.pw, iw = this.pu, o = k * 36, p = this.p, pi = this.pi;
    p[0] = w[o]; p[1] = w[o + 1]; p[2] = w[o + 2]; pi[0] = iw[o + 3];
    p[3] = w[o + 4]; p[4] = w[o + 5]; p[5] = w[o + 6]; pi[1] = iw[o + 7];
    pi[2] = iw[o + 8]; p[6] = w[o + 9];
    for (let i = 0; i < 12; i++) p[7 + i] = w[o + 10 + i];
  }

  store(k) {
    const w = this.pw, iw = this.pu, o = k * 36, p = this.p, pi = this.pi;
    w[o] = p[0]; w[o + 1] = p[1]; w[o + 2] = p[2]; iw[o + 3] = pi[0];
    w[o + 4] = p[3]; w[o + 5] = p[4]; w[o + 6] = p[5]; iw[o + 7] = pi[1];
    iw[o + 8] = pi[2]; w[o + 9] = p[6];
    for (let i = 0; i < 12; i++) w[o + 10 + i] = p[7 + i];
    for (let i = 0; i < 12; i++) w[o + 22 + i] = 1;  // transmittance (written, never read)
    iw[o + 34] = 0; iw[o + 35] = 0;
  }

  screen(x, y) {  // wgsl:118
    this.sx = F(fma32(F(x + 0.5), this.u.invRes[0], -0.5) * 2);
    this.sy = F(fma32(F(y + 0.5), this.u.invRes[1], -0.5) * -2);
  }

  // reset compute_main, wgsl:224-230 (full reset)
  resetRows(y0, y1) {
    const R = this.R;
    for (let y = y0; y < y1; y++) {
      for (let x = 0; x < R; x++) {
        this.screen(x, y);
        this.st = hash3(x, y, this.u.seedBits);
        this.reset(this.sx, this.sy);
        this.pi[1] = 0;
        for (let i = 0; i < 12; i++) this.p[7 + i] = 1;
        this.store(y * R + x);
      }
    }
  }

  // render compute_main for rows [y0, y1), wgsl:118-168
  renderRows(y0, y1, rgb32, rgba16) {
    const R = this.R, u = this.u, p = this.p, pi = this.pi, spec = this.spec;
    const smp = this.smp;
    const rcpExt = rcp(u.extinction);
    for (let y = y0; y < y1; y++) {
      for (let x = 0; x < R; x++) {
        this.screen(x, y);
        const sx = this.sx, sy = this.sy;
        const k = y * R + x;
        this.load(k);
        this.st = hash3(x, y, u.seedBits);
        for (let i = 0; i < u.steps; i++) {
          const dist = F(-specLog(this.uniform()) * rcpExt);  // exponential.wgsl
          p[0] = fma32(dist, p[3], p[0]);
          p[1] = fma32(dist, p[4], p[1]);
          p[2] = fma32(dist, p[5], p[2]);
          const dens = this.sampleVolume(p[0], p[1], p[2]);
          this.sampleTf(F(F(p[6] - 400) * rcp(300)), dens, smp);
          const albedo = smp[0], alpha = smp[1];
          const aniso = F(F(smp[2] * 2) - 1);
          const pnull = F(1 - alpha);
          const pscat = pi[0] >= u.maxBounces ? 0 : F(alpha * albedo);
          const pabs = F(F(1 - pnull) - pscat);
          const wheel = this.uniform();
          const oob = p[0] > 1 || p[1] > 1 || p[2] > 1 || p[0] < 0 || p[1] < 0 || p[2] < 0;
          if (oob) {
            const rad = this.sampleLight(p[3], p[4], p[5], p[6]);
            pi[1]++;
            this.addRadiance(rad);
            this.reset(sx, sy);
          } else if (wheel < pabs) {
            pi[1]++;
            this.addRadiance(0);
            this.reset(sx, sy);
          } else if (wheel < F(pabs + pscat)) {
            this.sampleHg(aniso);
            pi[0]++;
          }
        }
        this.store(k);
        // radiance_to_rgb, wgsl:304-326
        const nb = this.nBins();
        let X = 0, Y = 0, Z = 0;
        for (let b = 0; b < nb && b < 12; b++) {
          X = fma32(p[7 + b], spec[2 + nb + b], X);
          Y = fma32(p[7 + b], spec[2 + 2 * nb + b], Y);
          Z = fma32(p[7 + b], spec[2 + 3 * nb + b], Z);
        }
        const r = fma32(F(-0.498536), Z, fma32(F(-1.537150), Y, F(F(3.240479) * X)));
        const g = fma32(F(0.041556), Z, fma32(F(1.875990), Y, F(F(-0.969255) * X)));
        const bl = fma32(F(1.057311), Z, fma32(F(-0.204041), Y, F(F(0.055647) * X)));
        if (rgb32) { rgb32[k * 3] = r; rgb32[k * 3 + 1] = g; rgb32[k * 3 + 2] = bl; }
        if (rgba16) {
          rgba16[k * 4] = f2h(r); rgba16[k * 4 + 1] = f2h(g); rgba16[k * 4 + 2] = f2h(bl);
          rgba16[k * 4 + 3] = 0x3c00;
        }
      }
    }
  }

  sampleHg(g) {  // sampleHenyeyGreenstein, wgsl:82-97 (+ sphere.wgsl)
    const p = this.p, dk = this.dk;
    this.disk(dk);
    const nrm = fma32(dk[1], dk[1], F(dk[0] * dk[0]));
    const radius = F(2 * F(Math.sqrt(F(1 - nrm))));
    const ux = F(radius * dk[0]), uy = F(radius * dk[1]), uz = F(1 - F(2 * nrm));
    if (Math.abs(g) < EPS) { p[3] = ux; p[4] = uy; p[5] = uz; return; }
    const g2 = F(g * g);
    const c = F(F(1 - g2) * rcp(fma32(F(2 * g), this.uniform(), F(1 - g))));
    const hgcos = F(fma32(-c, c, F(1 + g2)) * rcp(F(2 * g)));
    const dx = p[3], dy = p[4], dz = p[5];
    const ud = dot3(ux, uy, uz, dx, dy, dz);
    const wx = fma32(-ud, dx, ux), wy = fma32(-ud, dy, uy), wz = fma32(-ud, dz, uz);
    const il = rcp(F(Math.sqrt(dot3(wx, wy, wz, wx, wy, wz))));
    const cx = F(wx * il), cy = F(wy * il), cz = F(wz * il);
    const sn = F(Math.sqrt(fma32(-hgcos, hgcos, 1)));
    p[3] = fma32(sn, cx, F(hgcos * dx));
    p[4] = fma32(sn, cy, F(hgcos * dy));
    p[5] = fma32(sn, cz, F(hgcos * dz));
  }
}

module.exports = { March, fma32, specLog, specSinCos, sc, pcg, hash3, f2h };
