// gamma.h -- device restatement of the pellet / gamma-ray / non-thermal-lepton states of update_packets
// (update_packets.cc:16-135, gammapkt.cc:227-700, photo_electric.cc, grey_emissivities.cc:12-77,
// nonthermal.cc:1877-1977, vectors.cc:10-44).  One packet per workitem; the arithmetic follows the reference's
// operation order (the engine is compiled with -ffp-contract=off) so that a packet's history matches the CPU
// oracle (oracle/oracle.cc, same sections) draw for draw.
//
// These states are short-lived (a pellet decays once, a gamma packet crosses a few dozen cells before it is
// absorbed or escapes) and end as k-packets, so they run in one grid-stride kernel (k_gamma, wavefront.h) at
// the start of each timestep's transport, ahead of the r-packet / macro-atom / k-packet rounds.
#ifndef ARTIS_GAMMA_H
#define ARTIS_GAMMA_H

#include "transport.h"

// pellet bookkeeping words of the packet record (packet.h:54-60), read-only on this path
struct PelletInfo {
  double tdecay;
  int originated;  // originated_from_particlenotgamma
  int decaytype;   // pellet_decaytype
};
DEVFN void pellet_info_load(const uint64_t *__restrict__ soa, int64_t n, int64_t i, PelletInfo &pi) {
  pi.tdecay = asd(soa[PW(n, i, 31)]);
  const uint64_t w = soa[PW(n, i, 34)];
  pi.originated = (int)(lo32(w) & 0xff);
  pi.decaytype = hi32(w);
}

DEVFN bool is_gamma_family(int type) {
  return type == ARTIS_TYPE_RADIOACTIVE_PELLET || type == ARTIS_TYPE_GAMMA || type == ARTIS_TYPE_NTLEPTON ||
         type == ARTIS_TYPE_NONTHERMAL_PREDEPOSIT;
}

// cell properties; the empty-cell sentinel mgi == npts_model reads as zero (grid.cc:840)
DEVFN double cell_rho(const Ctx &K, int mgi) { return mgi == K.G.npts_model ? 0. : (double)K.C.rho[mgi]; }
DEVFN double cell_nnetot(const Ctx &K, int mgi) { return mgi == K.G.npts_model ? 0. : (double)K.C.nnetot[mgi]; }
DEVFN double cell_ffegrp(const Ctx &K, int mgi) {
  return (mgi == K.G.npts_model || !K.C.ffegrp) ? 0. : (double)K.C.ffegrp[mgi];
}
DEVFN void vec_scale(double v[3], double s) {
  v[0] *= s;
  v[1] *= s;
  v[2] *= s;
}

// vectors.cc:10-44
DEVFN void scatter_dir(artis_rng *rng, const double dir_in[3], double cos_theta, double dir_out[3]) {
  const double zrand = artis_rng_uniform(rng);
  const double phi = zrand * 2 * ARTIS_PI;
  const double sin_theta_sq = 1. - (cos_theta * cos_theta);
  const double sin_theta = sqrt(sin_theta_sq);
  const double zprime = cos_theta;
  const double xprime = sin_theta * cos(phi);
  const double yprime = sin_theta * sin(phi);
  const double norm1 = 1. / sqrt((dir_in[0] * dir_in[0]) + (dir_in[1] * dir_in[1]));
  const double norm2 = 1. / sqrt((dir_in[0] * dir_in[0]) + (dir_in[1] * dir_in[1]) + (dir_in[2] * dir_in[2]));
  const double r11 = dir_in[1] * norm1;
  const double r12 = -1 * dir_in[0] * norm1;
  const double r13 = 0.0;
  const double r21 = dir_in[0] * dir_in[2] * norm1 * norm2;
  const double r22 = dir_in[1] * dir_in[2] * norm1 * norm2;
  const double r23 = -1 * norm2 / norm1;
  const double r31 = dir_in[0] * norm2;
  const double r32 = dir_in[1] * norm2;
  const double r33 = dir_in[2] * norm2;
  dir_out[0] = (r11 * xprime) + (r21 * yprime) + (r31 * zprime);
  dir_out[1] = (r12 * xprime) + (r22 * yprime) + (r32 * zprime);
  dir_out[2] = (r13 * xprime) + (r23 * yprime) + (r33 * zprime);
}

// gammapkt.cc:227-253
DEVFN void choose_gamma_ray(Tx &x, Pkt &p) {
  const Ctx &K = x.K;
  const int nucindex = p.pellet_nucindex;
  const double E_gamma = K.T.g_endecay[nucindex];
  const double zrand = artis_rng_uniform(&x.rng);
  const int off = K.T.g_off[nucindex];
  int nselected = -1;
  double runtot = 0.;
  for (int j = 0; j < K.T.g_nlines[nucindex]; j++) {
    runtot += K.T.g_prob[off + j] * K.T.g_energy[off + j] / E_gamma;
    if (zrand <= runtot) {
      nselected = j;
      break;
    }
  }
  if (nselected < 0) {
    x.err(ERR_GAMMA, p.number, 1);
    return;
  }
  p.nu_cmf = K.T.g_energy[off + nselected] / ARTIS_H;
}

// gammapkt.cc:255-313
DEVFN void pellet_gamma_decay(Tx &x, Pkt &p, const PelletInfo &pi) {
  const Ctx &K = x.K;
  if (p.pellet_nucindex < 0 || p.pellet_nucindex >= K.T.g_nnuc) {
    x.err(ERR_GAMMA, p.number, 2);
    return;
  }
  if (K.T.g_nlines[p.pellet_nucindex] == 0) {
    p.type = ARTIS_TYPE_KPKT;
    p.absorptiontype = -6;
    return;
  }
  double dir_cmf[3];
  get_rand_isotropic_unitvec(&x.rng, dir_cmf);
  const double t = -1. * pi.tdecay;
  const double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
  angle_ab(dir_cmf, vel_vec, p.dir);
  choose_gamma_ray(x, p);
  p.prop_time = pi.tdecay;
  const double dopplerfactor = doppler_packet(K, p);
  p.nu_rf = p.nu_cmf / dopplerfactor;
  p.e_rf = p.e_cmf / dopplerfactor;
  p.type = ARTIS_TYPE_GAMMA;
  p.last_cross = ARTIS_NONE;
  p.stokes[0] = 1.0;
  p.stokes[1] = p.stokes[2] = 0.0;
  double dummy_dir[3] = {0., 0., 1.};
  cross_prod(p.dir, dummy_dir, p.pol_dir);
  if ((dot(p.pol_dir, p.pol_dir)) < 1.e-8) {
    dummy_dir[0] = dummy_dir[2] = 0.0;
    dummy_dir[1] = 1.0;
    cross_prod(p.dir, dummy_dir, p.pol_dir);
  }
  vec_norm(p.pol_dir, p.pol_dir);
}

// gammapkt.cc:315-326
DEVFN double sigma_compton_partial(double x, double f) {
  const double term1 = ((x * x) - (2 * x) - 2) * log(f) / x / x;
  const double term2 = (((f * f) - 1) / (f * f)) / 2;
  const double term3 = ((f - 1) / x) * ((1 / x) + (2 / f) + (1 / (x * f)));
  return (3 * ARTIS_SIGMA_T * (term1 + term2 + term3) / (8 * x));
}

// gammapkt.cc:328-354
DEVFN double sig_comp(const Ctx &K, const Pkt &p) {
  const double xx = ARTIS_H * p.nu_cmf / ARTIS_ME / ARTIS_CLIGHT / ARTIS_CLIGHT;
  double sigma_cmf;
  if (xx < ARTIS_THOMSON_LIMIT) {
    sigma_cmf = ARTIS_SIGMA_T;
  } else {
    const double fmax = (1 + (2 * xx));
    sigma_cmf = sigma_compton_partial(xx, fmax);
  }
  sigma_cmf *= cell_nnetot(K, cell_mgi(K, p.where));
  return sigma_cmf * doppler_packet(K, p);
}

// gammapkt.cc:356-397 (bisection, at most 1000 halvings)
DEVFN double choose_f(double xx, double zrand) {
  double f_max = 1 + (2 * xx);
  double f_min = 1;
  const double norm = zrand * sigma_compton_partial(xx, f_max);
  int count = 0;
  double err = 1e20;
  double ftry = (f_max + f_min) / 2;
  while ((err > 1.e-4) && (count < 1000)) {
    ftry = (f_max + f_min) / 2;
    const double sigma_try = sigma_compton_partial(xx, ftry);
    if (sigma_try > norm) {
      f_max = ftry;
      err = (sigma_try - norm) / norm;
    } else {
      f_min = ftry;
      err = (norm - sigma_try) / norm;
    }
    count++;
  }
  return ftry;
}

// gammapkt.cc:399-420
DEVFN double thomson_angle(Tx &x, const Pkt &p) {
  const double zrand = artis_rng_uniform(&x.rng);
  const double B_coeff = (8. * zrand) - 4.;
  double t_coeff = sqrt((B_coeff * B_coeff) + 4);
  t_coeff = t_coeff - B_coeff;
  t_coeff = t_coeff / 2;
  t_coeff = cbrt(t_coeff);
  const double mu = (1 / t_coeff) - t_coeff;
  if (fabs(mu) > 1) x.err(ERR_GAMMA, p.number, 3);
  return mu;
}

// gammapkt.cc:422-531
DEVNI void compton_scatter(Tx &x, Pkt &p) {
  const Ctx &K = x.K;
  double f;
  const double xx = ARTIS_H * p.nu_cmf / ARTIS_ME / ARTIS_CLIGHT / ARTIS_CLIGHT;
  bool stay_gamma;
  if (xx < ARTIS_THOMSON_LIMIT) {
    f = 1.0;
    stay_gamma = true;
  } else {
    const double zrand = artis_rng_uniform(&x.rng);
    f = choose_f(xx, zrand);
    if ((f < 1) || (f > (2 * xx + 1))) {
      x.err(ERR_GAMMA, p.number, 4);
      return;
    }
    const double prob_gamma = 1. / f;
    const double zrand2 = artis_rng_uniform(&x.rng);
    stay_gamma = (zrand2 < prob_gamma);
  }
  if (stay_gamma) {
    p.nu_cmf = p.nu_cmf / f;
    const double t = p.prop_time;
    double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
    double cmf_dir[3];
    angle_ab(p.dir, vel_vec, cmf_dir);
    double cos_theta;
    if (xx < ARTIS_THOMSON_LIMIT)
      cos_theta = thomson_angle(x, p);
    else
      cos_theta = 1. - ((f - 1) / xx);
    double new_dir[3];
    scatter_dir(&x.rng, cmf_dir, cos_theta, new_dir);
    const double test = dot(new_dir, new_dir);
    if (fabs(1. - test) > 1.e-8) x.err(ERR_GAMMA, p.number, 5);
    const double test2 = dot(new_dir, cmf_dir);
    if (fabs(test2 - cos_theta) > 1.e-8) x.err(ERR_GAMMA, p.number, 6);
    vec_scale(vel_vec, -1.);
    double final_dir[3];
    angle_ab(new_dir, vel_vec, final_dir);
    for (int d = 0; d < 3; d++) p.dir[d] = final_dir[d];
    const double dopplerfactor = doppler_packet(K, p);
    p.nu_rf = p.nu_cmf / dopplerfactor;
    p.e_rf = p.e_cmf / dopplerfactor;
    p.last_cross = ARTIS_NONE;
  } else {
    p.type = ARTIS_TYPE_NTLEPTON;
    p.absorptiontype = -3;
    lctr(x.L, CTR_NT_STAT_FROM_GAMMA);
  }
}

// photo_electric.cc:10-48
DEVFN double sig_photo_electric(const Ctx &K, const Pkt &p) {
  double sigma_cmf;
  const int mgi = cell_mgi(K, p.where);
  const double rho = cell_rho(K, mgi);
  if (K.R.gamma_grey < 0) {
    double sigma_cmf_si = 1.16e-24 * pow(p.nu_cmf / 2.41326e19, -3.13);
    double sigma_cmf_fe = 25.7e-24 * pow(p.nu_cmf / 2.41326e19, -3.0);
    sigma_cmf_si *= rho / ARTIS_MH / 28;
    sigma_cmf_fe *= rho / ARTIS_MH / 56;
    const double f_fe = cell_ffegrp(K, mgi);
    sigma_cmf = (sigma_cmf_fe * f_fe) + (sigma_cmf_si * (1. - f_fe));
  } else {
    sigma_cmf = K.R.gamma_grey * rho;
  }
  return sigma_cmf * doppler_packet(K, p);
}

// photo_electric.cc:50-111
DEVFN double sig_pair_prod(const Ctx &K, const Pkt &p) {
  double sigma_cmf;
  const int mgi = cell_mgi(K, p.where);
  const double rho = cell_rho(K, mgi);
  if (K.R.gamma_grey < 0) {
    if (p.nu_cmf > 2.46636e+20) {
      double sigma_cmf_si;
      double sigma_cmf_fe;
      const double f_fe = cell_ffegrp(K, mgi);
      if (p.nu_cmf > 3.61990e+20) {
        sigma_cmf_si = (0.0481 + (0.301 * ((p.nu_cmf / 2.41326e+20) - 1.5))) * 196.e-27;
        sigma_cmf_fe = (0.0481 + (0.301 * ((p.nu_cmf / 2.41326e+20) - 1.5))) * 784.e-27;
      } else {
        sigma_cmf_si = 1.0063 * ((p.nu_cmf / 2.41326e+20) - 1.022) * 196.e-27;
        sigma_cmf_fe = 1.0063 * ((p.nu_cmf / 2.41326e+20) - 1.022) * 784.e-27;
      }
      sigma_cmf_si *= rho / ARTIS_MH / 28;
      sigma_cmf_fe *= rho / ARTIS_MH / 56;
      sigma_cmf = (sigma_cmf_fe * f_fe) + (sigma_cmf_si * (1. - f_fe));
    } else {
      sigma_cmf = 0.0;
    }
  } else {
    sigma_cmf = 0.0;
  }
  double sigma_rf = sigma_cmf * doppler_packet(K, p);
  if (sigma_rf < 0) sigma_rf = 0.0;
  return sigma_rf;
}

// photo_electric.cc:113-166
DEVNI void pair_prod(Tx &x, Pkt &p) {
  const Ctx &K = x.K;
  const double prob_gamma = 1.022 * ARTIS_MEV / (ARTIS_H * p.nu_cmf);
  if (prob_gamma < 0) {
    x.err(ERR_GAMMA, p.number, 7);
    return;
  }
  const double zrand = artis_rng_uniform(&x.rng);
  if (zrand > prob_gamma) {
    p.type = ARTIS_TYPE_NTLEPTON;
    p.absorptiontype = -5;
    lctr(x.L, CTR_NT_STAT_FROM_GAMMA);
  } else {
    p.nu_cmf = 0.511 * ARTIS_MEV / ARTIS_H;
    double dir_cmf[3];
    get_rand_isotropic_unitvec(&x.rng, dir_cmf);
    const double t = -1. * p.prop_time;
    const double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
    angle_ab(dir_cmf, vel_vec, p.dir);
    const double dopplerfactor = doppler_packet(K, p);
    p.nu_rf = p.nu_cmf / dopplerfactor;
    p.e_rf = p.e_cmf / dopplerfactor;
    p.type = ARTIS_TYPE_GAMMA;
    p.last_cross = ARTIS_NONE;
  }
}

// grey_emissivities.cc:12-26
DEVFN double meanf_sigma(double x) {
  double f = 1 + (2 * x);
  double term0 = 2 / x;
  double term1 = (1 - (2 / x) - (3 / (x * x))) * log(f);
  double term2 = ((4 / x) + (3 / (x * x)) - 1) * 2 * x / f;
  double term3 = (1 - (2 / x) - (1 / (x * x))) * 2 * x * (1 + x) / f / f;
  double term4 = -2. * x * ((4 * x * x) + (6 * x) + 3) / 3 / f / f / f;
  double tot = 3 * ARTIS_SIGMA_T * (term0 + term1 + term2 + term3 + term4) / (8 * x);
  return tot;
}

// grey_emissivities.cc:28-77
DEVFN void rlc_emiss_gamma(const Ctx &K, const Pkt &p, double dist) {
  const int mgi = cell_mgi(K, p.where);
  if (dist > 0) {
    const double t = p.prop_time;
    const double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
    const double xx = ARTIS_H * p.nu_cmf / ARTIS_ME / ARTIS_CLIGHT / ARTIS_CLIGHT;
    double heating_cont = ((meanf_sigma(xx) * cell_nnetot(K, mgi)) + sig_photo_electric(K, p) +
                           (sig_pair_prod(K, p) * (1. - (2.46636e+20 / p.nu_cmf))));
    heating_cont = heating_cont * p.e_rf * dist * (1. - (2. * dot(vel_vec, p.dir) / ARTIS_CLIGHT));
    safeadd(&K.E.rpkt_emiss[mgi], 1.e-20 * heating_cont);
  }
}

// get_nul (gammapkt.cc:720-745): the index of the line of allnuc_gamma_line_list to the red of freq
#define GAMMA_RED_OF_LIST (-956)  // gammapkt.cc:33
DEVFN int get_nul(const Ctx &K, double freq) {
  const double *f = K.T.g_freq_sorted;
  const int n = K.T.g_nsorted;
  if (n < 1) return GAMMA_RED_OF_LIST;  // (no gamma-ray lines: no gamma packets either)
  if (freq > f[n - 1]) return n - 1;
  if (freq < f[0]) return GAMMA_RED_OF_LIST;
  // one line and freq == f[0]: the reference's bisection below never ends (too_high == too_low == 0); the line
  // itself is the one to the red
  if (n == 1) return 0;
  int too_high = n - 1, too_low = 0;
  while (too_high != too_low + 1) {
    const int tryindex = (too_high + too_low) / 2;
    if (f[tryindex] >= freq)
      too_high = tryindex;
    else
      too_low = tryindex;
  }
  return too_low;
}

// compton_emiss_cont (emissivities.cc:14-113): the Compton emissivity towards syn_dir of a gamma packet about to
// travel dist, binned by the gamma-ray line to the red of the scattered frequency
DEVNI void compton_emiss_cont(Tx &x, const Pkt &p, double dist) {
  const Ctx &K = x.K;
  const double t = p.prop_time;
  const double vel_vec[3] = {p.pos[0] / t, p.pos[1] / t, p.pos[2] / t};
  double cmf_dir[3], cmf_syn_dir[3];
  angle_ab(p.dir, vel_vec, cmf_dir);
  angle_ab(K.R.syn_dir, vel_vec, cmf_syn_dir);
  const double mu_cmf = dot(cmf_dir, cmf_syn_dir);
  if (mu_cmf > 1 || mu_cmf < -1) {  // "problem with Compton emissivity. Abort."
    x.err(ERR_GAMMA, p.number, 20);
    return;
  }
  const double f = 1 + (ARTIS_H * p.nu_cmf / ARTIS_ME / ARTIS_CLIGHT / ARTIS_CLIGHT * (1. - mu_cmf));
  const double freq_out = p.nu_cmf / f;
  const int lindex = get_nul(K, freq_out);
  if ((lindex > K.R.emiss_offset - 1) && (lindex < K.R.emiss_offset + K.R.emiss_max - 1)) {
    const double dsigma_domega_cmf = 0.0596831 * ARTIS_SIGMA_T / f / f * (f + (1. / f) + (mu_cmf * mu_cmf) - 1.);
    const double dop_fac = doppler_pos_dir(K, p.pos, p.dir, p.prop_time);  // doppler_nucmf_on_nurf(dir, vel_vec)
    const double emiss_cont = p.e_rf * dsigma_domega_cmf * dist * dop_fac * dop_fac / f;
    if (lindex >= K.R.emiss_offset)  // (below: the reference's "scarily bad error" printout, nothing added)
      safeadd(&K.E.compton[(int64_t)cell_mgi(K, p.where) * ARTIS_EMISS_MAX + lindex - K.R.emiss_offset], emiss_cont);
  }
}

// pp_emiss_cont (emissivities.cc:115-136): pair-production emissivity in the last emissivity slot
DEVFN void pp_emiss_cont(const Ctx &K, const Pkt &p, double dist) {
  const double emiss_cont = sig_pair_prod(K, p) * (2.46636e+20 / p.nu_cmf) * p.e_rf * dist;
  safeadd(&K.E.compton[(int64_t)cell_mgi(K, p.where) * ARTIS_EMISS_MAX + K.R.emiss_max - 1], 1.e-20 * emiss_cont);
}

// the estimators of one path segment of do_gamma (gammapkt.cc:618-625, 639-646, 653-660)
DEVFN void gamma_segment_estimators(Tx &x, const Pkt &p, double dist, double kap_tot) {
  if (kap_tot > 0) {
    if (x.K.R.comp_est_now) {
      compton_emiss_cont(x, p, dist);
      pp_emiss_cont(x.K, p, dist);
    }
    if (x.K.R.do_rlc_est != 0) rlc_emiss_gamma(x.K, p, dist);
  }
}

// gammapkt.cc:533-700: one step of a gamma packet (cell boundary, end of the timestep or an interaction)
DEVNI void do_gamma(Tx &x, Pkt &p, double t2) {
  const Ctx &K = x.K;
  double zrand = artis_rng_uniform_pos(&x.rng);
  const double tau_next = -1. * log(zrand);
  const double tau_current = 0.0;
  int snext = -1;
  double sdist = boundary_cross(x, p, &snext);
  const double maxsdist = max_sdist(K, p, sdist);
  if (sdist > maxsdist) {
    x.err(ERR_SDIST, p.number, p.where);
    return;
  }
  if (sdist < 0) sdist = 0;
  if (((snext < 0) && (snext != -99)) || (snext >= K.G.ngrid)) {
    x.err(ERR_BADCELL, p.number, snext);
    return;
  }
  if (sdist > K.R.max_path_step) {
    sdist = K.R.max_path_step;
    snext = p.where;
  }
  double kap_compton = 0.0;
  if (K.R.gamma_grey < 0) kap_compton = sig_comp(K, p);
  const double kap_photo_electric = sig_photo_electric(K, p);
  const double kap_pair_prod = sig_pair_prod(K, p);
  const double kap_tot = kap_compton + kap_photo_electric + kap_pair_prod;
  const double edist = (tau_next - tau_current) / kap_tot;
  if (edist < 0) {
    x.err(ERR_EDIST, p.number, 10);
    return;
  }
  const double tdist = (t2 - p.prop_time) * ARTIS_CLIGHT_PROP;
  if (tdist < 0) {
    x.err(ERR_EDIST, p.number, 11);
    return;
  }
  if ((sdist < tdist) && (sdist < edist)) {
    p.prop_time += sdist / 2. / ARTIS_CLIGHT_PROP;
    move_pkt(K, p, sdist / 2.);
    gamma_segment_estimators(x, p, sdist, kap_tot);
    p.prop_time += sdist / 2. / ARTIS_CLIGHT_PROP;
    move_pkt(K, p, sdist / 2.);
    if (snext != p.where) change_cell(x, p, snext);
  } else if ((tdist < sdist) && (tdist < edist)) {
    p.prop_time += tdist / 2. / ARTIS_CLIGHT_PROP;
    move_pkt(K, p, tdist / 2.);
    gamma_segment_estimators(x, p, tdist, kap_tot);
    p.prop_time = t2;
    move_pkt(K, p, tdist / 2.);
  } else if ((edist < sdist) && (edist < tdist)) {
    p.prop_time += edist / 2. / ARTIS_CLIGHT_PROP;
    move_pkt(K, p, edist / 2.);
    gamma_segment_estimators(x, p, edist, kap_tot);
    p.prop_time += edist / 2. / ARTIS_CLIGHT_PROP;
    move_pkt(K, p, edist / 2.);
    zrand = artis_rng_uniform(&x.rng);
    if (kap_compton > (zrand * kap_tot)) {
      compton_scatter(x, p);
    } else if ((kap_compton + kap_photo_electric) > (zrand * kap_tot)) {
      p.type = ARTIS_TYPE_NTLEPTON;
      p.absorptiontype = -4;
      lctr(x.L, CTR_NT_STAT_FROM_GAMMA);
    } else if ((kap_compton + kap_photo_electric + kap_pair_prod) > (zrand * kap_tot)) {
      pair_prod(x, p);
    } else {
      x.err(ERR_NOEVENT, p.number, 10);
    }
  } else {
    x.err(ERR_NOEVENT, p.number, 11);
  }
}

// update_packets.cc:16-69
DEVFN void do_nonthermal_predeposit(Tx &x, Pkt &p, const PelletInfo &pi, double t2) {
  const Ctx &K = x.K;
  const double ts = p.prop_time;
  const double particle_en = ARTIS_H * p.nu_cmf;
  double endot = 0.;
  double t_absorb = ts;
  if (!K.R.instant_particle_deposition) {
    const double rho = cell_rho(K, cell_mgi(K, p.where));
    endot = (pi.decaytype == ARTIS_DECAYTYPE_ALPHA) ? 5.e11 * ARTIS_MEV * rho : 4.e10 * ARTIS_MEV * rho;
    const double zrand = artis_rng_uniform(&x.rng);
    const double en_absorb = zrand * particle_en;
    t_absorb = ts + en_absorb / endot;
  }
  if (t_absorb <= t2) {
    if (pi.decaytype == ARTIS_DECAYTYPE_ALPHA)
      safeadd(&K.E.scalars[5], p.e_cmf);  // alpha_dep
    else if (pi.decaytype == ARTIS_DECAYTYPE_BETAMINUS)
      safeadd(&K.E.scalars[3], p.e_cmf);  // electron_dep
    else if (pi.decaytype == ARTIS_DECAYTYPE_BETAPLUS)
      safeadd(&K.E.scalars[2], p.e_cmf);  // positron_dep
    vec_scale(p.pos, t_absorb / ts);
    p.prop_time = t_absorb;
    p.type = ARTIS_TYPE_NTLEPTON;
  } else {
    p.nu_cmf = (particle_en - endot * (t2 - ts)) / ARTIS_H;
    vec_scale(p.pos, t2 / ts);
    p.prop_time = t2;
  }
}

// update_packets.cc:71-135
DEVFN void update_pellet(Tx &x, Pkt &p, const PelletInfo &pi, double t2) {
  const Ctx &K = x.K;
  const double ts = p.prop_time;
  const double tdecay = pi.tdecay;
  if (tdecay > t2) {
    vec_scale(p.pos, t2 / ts);
    p.prop_time = t2;
  } else if (tdecay > ts) {
    safeadd(&K.E.scalars[9], 1.);  // time_step[nts].pellet_decays
    p.prop_time = tdecay;
    vec_scale(p.pos, tdecay / ts);
    if (pi.originated) {
      if (pi.decaytype == ARTIS_DECAYTYPE_BETAPLUS) {
        safeadd(&K.E.scalars[2], p.e_cmf);  // positron_dep
        p.type = ARTIS_TYPE_NTLEPTON;
        p.absorptiontype = -10;
      } else if (pi.decaytype == ARTIS_DECAYTYPE_BETAMINUS) {
        safeadd(&K.E.scalars[4], p.e_cmf);  // electron_emission
        p.em_time = (int)p.prop_time;
        p.type = ARTIS_TYPE_NONTHERMAL_PREDEPOSIT;
        p.absorptiontype = -10;
      } else if (pi.decaytype == ARTIS_DECAYTYPE_ALPHA) {
        safeadd(&K.E.scalars[6], p.e_cmf);  // alpha_emission
        p.em_time = (int)p.prop_time;
        p.type = ARTIS_TYPE_NONTHERMAL_PREDEPOSIT;
        p.absorptiontype = -10;
      }
    } else {
      safeadd(&K.E.scalars[7], p.e_cmf);  // gamma_emission
      pellet_gamma_decay(x, p, pi);
    }
  } else if ((tdecay > 0) && (x.nts == 0)) {
    p.e_cmf *= tdecay / K.G.tmin;
    p.type = ARTIS_TYPE_PRE_KPKT;
    p.absorptiontype = -7;
    lctr(x.L, CTR_K_STAT_FROM_EARLIERDECAY);
    p.prop_time = K.G.tmin;
  } else {
    x.err(ERR_GAMMA, p.number, 8);
  }
}

// nonthermal.cc:1877-1977 (NT_EXCITATION_ON false): with NT_ON && NT_SOLVE_SPENCERFANO outside thick cells the
// fraction frac_ionization = get_ntion_energyrate / deposition_rate_density activates a macro-atom by non-thermal
// ionisation (select_nt_ionization2 over the per-cell running sums of k_ntcells, then the Auger upper ion); the
// rest, and every deposition without the Spencer-Fano solution, becomes a k-packet
DEVFN void do_ntlepton(Tx &x, Pkt &p) {
  const Ctx &K = x.K;
  safeadd(&K.E.scalars[8], p.e_cmf);  // nt_energy_deposited
  const int mgi = cell_mgi(K, p.where);
  if (K.R.nt_on && K.R.nt_solve_spencerfano && K.C.thick[mgi] != 1) {
    const int k = K.C.ne_index[mgi];
    const double zrand = artis_rng_uniform(&x.rng);
    const double ratetotal = K.C.nt_total[k];
    const double frac_ionization = ratetotal / K.C.nt_dep[mgi];
    if (zrand < frac_ionization) {
      const double z2 = artis_rng_uniform(&x.rng);
      const double *cum = K.C.nt_cum + (int64_t)k * K.T.nions_total;
      int element = -1, lowerion = -1;
      for (int e = 0; e < K.T.nelements && element < 0; e++)
        for (int li = 0; li < K.T.elem_nions[e] - 1; li++)
          if (cum[uion(K, e, li)] >= z2 * ratetotal) {
            element = e;
            lowerion = li;
            break;
          }
      const int upperion = element < 0 ? -1 : nt_random_upperion(K, x.rng, mgi, element, lowerion, true);
      if (upperion < 0) {
        x.err(ERR_MA_SELECT, p.number, 20);
        return;
      }
      p.ma_element = element;
      p.ma_ion = upperion;
      p.ma_level = 0;
      p.ma_activatingline = -99;
      p.type = ARTIS_TYPE_MA;
      lctr(x.L, CTR_MA_STAT_ACTIVATION_NTCOLLION);
      p.interactions += 1;
      p.last_event = 20;
      p.trueemissiontype = -1;
      p.trueemissionvelocity = -1;
      lctr(x.L, CTR_NT_STAT_TO_IONIZATION);
      return;
    }
  }
  p.last_event = 22;
  p.type = ARTIS_TYPE_KPKT;
  lctr(x.L, CTR_NT_STAT_TO_KPKT);
}

// update_packets.cc:137-170: one do_packet call for a packet of the gamma family
DEVFN void do_gamma_family_step(Tx &x, Pkt &p, const PelletInfo &pi, double t2) {
  const Ctx &K = x.K;
  switch (p.type) {
    case ARTIS_TYPE_RADIOACTIVE_PELLET:
      update_pellet(x, p, pi, t2);
      break;
    case ARTIS_TYPE_GAMMA:
      do_gamma(x, p, t2);
      if (p.type != ARTIS_TYPE_GAMMA && p.type != ARTIS_TYPE_ESCAPE) safeadd(&K.E.scalars[1], p.e_cmf);  // gamma_dep
      break;
    case ARTIS_TYPE_NONTHERMAL_PREDEPOSIT:
      do_nonthermal_predeposit(x, p, pi, t2);
      break;
    case ARTIS_TYPE_NTLEPTON:
      do_ntlepton(x, p);
      break;
    default:
      x.err(ERR_UNSUPPORTED_TYPE, p.number, p.type);
  }
}

#endif
