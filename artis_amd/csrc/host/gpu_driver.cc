// gpu_driver.cc -- a C++ host that drives the engine the way sn3d.cc's timestep loop does (sn3d.cc:540-650):
// per timestep update_grid (here: the synthetic LTE stand-in) -> upload_cellstate -> zero_estimators ->
// update_packets -> write the raw packet file.  It exercises the C++ mirror (update_packets_gpu.h) without
// Python.  Usage:
//   artis_gpu_driver <outdir> <ngrid> <nlevels_per_ion> <n_ionising> <max_lines> <ntstep> <nts0> <nsteps>
//                    <npkts> <seed> [<gamma_lines_dir>]
// With <gamma_lines_dir> (holding ni56_lines.txt / co56_lines.txt, the reference's data/ files) the run starts
// from radioactive pellets at tmin (packet_init, packet.cc:59-149) instead of r-packets.
// Writes <outdir>/packets_0000_ts<nts>.tmp (raw 304-byte records, sn3d.cc:387-398) after every timestep, the
// final <outdir>/packets00_0000.out (packet.cc:152-196), and prints one summary line per timestep.
// ARTIS_DRIVER_RCCL=1: the estimators go through the RCCL all-reduce of update_packets_reduced (a
// communicator of this one rank -- the multi-rank host hands rank 0's id to every rank).
// ARTIS_DRIVER_TE=1: after the last timestep, update_grid's temperature / ionisation solution on the GPU
// (PacketEngine::solve_temperatures) from that timestep's own estimators, normalised as update_grid.cc:1041-1150
// does (see te_from_estimators); inputs and outputs go to <outdir>/te_case.bin for the oracle replay in
// tests/test_host_driver.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "artis_io.h"
#include "artis_layout_check.h"
#include "model_synth.h"
#include "update_packets_gpu.h"


namespace {
// One artis_te_cells block built from a timestep's raw estimators, as update_grid_cell prepares them
// (update_grid.cc:1041-1150): estimator_normfactor = 1 / deltaV / deltat / nprocs; J, nuJ normalised with an extra
// 1/4pi (radfield::normalise_J / normalise_nuJ); T_J = (pi J / sigma)^(1/4), T_R = h nubar / k / 3.832229494 and
// W = pi J / sigma / T_R^4, each clamped to [MINTEMP, MAXTEMP] (radfield.cc:1136-1175, set_params_fullspec);
// ff / collisional heating times the factor (update_grid.cc:1133-1134); the bf-heating estimator times the factor
// over the ground level's analytic coefficient (update_grid.cc:950-960).  Stand-ins where the reference needs data
// this synthetic model does not carry: Gamma per ground-level population = gammaestimator * factor / h (the
// reference's calculate_iongamma_per_gspop sums the corrected photoionisation coefficients), mean atomic weight
// 2.1 Z m_H, and vol_init from the uniform grid's cell count per model cell.
struct TeCase {
  std::vector<int32_t> mgi;
  std::vector<float> TR, W, TJ, rho, abund, meanw, Te, gp, nne, nnetot, pf;
  std::vector<int16_t> thick;
  std::vector<double> vol, ff, col, gam, bfh, totcool, ccion, rates;
  std::vector<int32_t> iters;
  artis_te_cells cells{};
  artis_te_params par{};
};
void te_from_estimators(const artis_atomic_tables &at, const artis_geometry &g, const artis_cell_state &cs,
                        const artis_te_tables &tab, int nts, int np, const std::vector<double> &J,
                        const std::vector<double> &nuJ, const std::vector<double> &ff,
                        const std::vector<double> &col, const std::vector<double> &gam,
                        const std::vector<double> &bfh, TeCase &c) {
  const int nel = at.nelements, ni = at.nions_total, mx = at.maxnions;
  const double PI = 3.14159265358979323846, STEBO = 5.670400e-5, H = 6.6260755e-27, KB = 1.38064852e-16,
               MH = 1.67352e-24;
  const double T_step_log = (std::log(at.maxtemp) - std::log(at.mintemp)) / (at.tablesize - 1.);
  std::vector<int> count(np + 1, 0);
  for (int i = 0; i < g.ngrid; i++) count[g.cell_mgi[i]]++;
  const double wid = 2 * g.coordmax[0] / g.ncoordgrid[0];
  c.TR.assign(cs.TR, cs.TR + np);
  c.W.assign(cs.W, cs.W + np);
  c.TJ.assign(cs.TJ, cs.TJ + np);
  c.rho.assign(cs.rho, cs.rho + np);
  c.thick.assign(cs.thick, cs.thick + np);
  c.abund.assign(cs.elem_abundance, cs.elem_abundance + (size_t)np * nel);
  c.Te.assign(cs.Te, cs.Te + np);
  c.gp.assign(cs.groundlevelpop, cs.groundlevelpop + (size_t)np * ni);
  c.meanw.resize((size_t)np * nel);
  c.vol.resize(np);
  c.ff.assign(np, 0.);
  c.col.assign(np, 0.);
  c.gam.assign((size_t)np * nel * mx, 0.);
  c.bfh.assign((size_t)np * nel * mx, 1.);
  const double tmid = g.ts_mid[nts], deltat = g.ts_width[nts];
  for (int mgi = 0; mgi < np; mgi++) {
    for (int e = 0; e < nel; e++) c.meanw[(size_t)mgi * nel + e] = (float)(2.1 * at.elem_anumber[e] * MH);
    c.vol[mgi] = wid * wid * wid * count[mgi];
    if (!(c.rho[mgi] > 0) || count[mgi] == 0) continue;
    c.mgi.push_back(mgi);
    const double deltaV = c.vol[mgi] * std::pow(tmid / g.tmin, 3);
    const double normfactor = 1. / deltaV / deltat / 1;
    const double Jn = J[mgi] * normfactor / (4 * PI), nuJn = nuJ[mgi] * normfactor / (4 * PI);
    const double nubar = nuJn / Jn;
    if (std::isfinite(nubar) && nubar != 0.) {
      float T_J = std::pow(Jn * PI / STEBO, 1 / 4.);
      T_J = std::min<float>(std::max<float>(T_J, at.mintemp), at.maxtemp);
      float T_R = H * nubar / KB / 3.832229494;
      T_R = std::min<float>(std::max<float>(T_R, at.mintemp), at.maxtemp);
      c.TJ[mgi] = T_J;
      c.TR[mgi] = T_R;
      c.W[mgi] = Jn * PI / STEBO / std::pow(T_R, 4);
    }
    c.ff[mgi] = ff[mgi] * normfactor;
    c.col[mgi] = col[mgi] * normfactor;
    for (int e = 0; e < nel; e++)
      for (int i = 0; i < at.elem_nions[e] - 1; i++) {
        const size_t ix = (size_t)mgi * nel * mx + e * mx + i;
        c.gam[ix] = gam[ix] * normfactor / H;
        // thermalbalance.cc:34-57 get_bfheatingcoeff_ana for (ion, level 0, target 0) at this cell's T_R, W
        const int ul = at.ion_uniqueleveloffset[at.elem_uniqueionoffset[e] + i];
        if (at.level_nphixstargets[ul] <= 0) continue;
        const int contindex = -1 - at.level_cont_index[ul];
        const double T = c.TR[mgi];
        const int lo = (int)std::floor(std::log(T / at.mintemp) / T_step_log);
        double coeff;
        if (lo < at.tablesize - 1) {
          const double Tl = at.mintemp * std::exp(lo * T_step_log), Tu = at.mintemp * std::exp((lo + 1) * T_step_log);
          const double fl = tab.bfheating_coeff[(size_t)lo * at.nbfcontinua + contindex];
          const double fu = tab.bfheating_coeff[(size_t)(lo + 1) * at.nbfcontinua + contindex];
          coeff = fl + (fu - fl) / (Tu - Tl) * (T - Tl);
        } else {
          coeff = tab.bfheating_coeff[(size_t)(at.tablesize - 1) * at.nbfcontinua + contindex];
        }
        coeff *= c.W[mgi];
        const double v = bfh[ix] * normfactor / coeff;
        c.bfh[ix] = (std::isfinite(v) && v > 0.) ? v : 1.;
      }
  }
  c.nne.assign(np, 0.f);
  c.nnetot.assign(np, 0.f);
  c.pf.assign((size_t)np * ni, 0.f);
  c.totcool.assign(np, 0.);
  c.ccion.assign((size_t)np * ni, 0.);
  c.rates.assign((size_t)np * ARTIS_TE_NRATES, 0.);
  c.iters.assign(np, 0);
  artis_te_cells &x = c.cells;
  x.ncells = (int32_t)c.mgi.size();
  x.mgi = c.mgi.data();
  x.TR = c.TR.data();
  x.W = c.W.data();
  x.TJ = c.TJ.data();
  x.rho = c.rho.data();
  x.thick = c.thick.data();
  x.elem_abundance = c.abund.data();
  x.elem_meanweight = c.meanw.data();
  x.vol_init = c.vol.data();
  x.ffheatingestimator = c.ff.data();
  x.colheatingestimator = c.col.data();
  x.gammaestimator = c.gam.data();
  x.bfheatingestimator = c.bfh.data();
  x.heating_dep = nullptr;
  x.Te = c.Te.data();
  x.groundlevelpop = c.gp.data();
  x.nne = c.nne.data();
  x.nnetot = c.nnetot.data();
  x.partfunct = c.pf.data();
  x.totalcooling = c.totcool.data();
  x.cooling_contrib_ion = c.ccion.data();
  x.heatingcoolingrates = c.rates.data();
  x.te_iterations = c.iters.data();
  c.par.t_current = tmid;
  c.par.tmin = g.tmin;
  c.par.T_min = at.mintemp;
  c.par.T_max = at.maxtemp;
  c.par.accuracy = 1e-2;  // TEMPERATURE_SOLVER_ACCURACY (artisoptions_classic.h:199)
  c.par.initial_iteration = 0;
}
template <typename T>
void put(std::ofstream &o, const std::vector<T> &v) {
  const int64_t n = (int64_t)v.size();
  o.write((const char *)&n, sizeof n);
  o.write((const char *)v.data(), (std::streamsize)(v.size() * sizeof(T)));
}
}  // namespace

int main(int argc, char **argv) {
  if (argc != 11 && argc != 12) {
    std::fprintf(stderr,
                 "usage: %s outdir ngrid nlevels_per_ion n_ionising max_lines ntstep nts0 nsteps npkts seed "
                 "[gamma_lines_dir]\n",
                 argv[0]);
    return 2;
  }
  const bool pellets = argc == 12;
  const std::string outdir = argv[1];
  artis_synth_config cfg;
  artis_synth_default_config(&cfg);
  cfg.ngrid_1d = std::atoi(argv[2]);
  cfg.nlevels_per_ion = std::atoi(argv[3]);
  cfg.n_ionising = std::atoi(argv[4]);
  cfg.max_lines = std::atoi(argv[5]);
  cfg.ntstep = std::atoi(argv[6]);
  const int nts0 = std::atoi(argv[7]), nsteps = std::atoi(argv[8]), npkts = std::atoi(argv[9]);
  const uint64_t seed = std::strtoull(argv[10], nullptr, 10);

  artis_model *m = artis_model_synth(&cfg);
  if (!m) {
    std::fprintf(stderr, "model synthesis failed\n");
    return 1;
  }
  const artis_atomic_tables &at = *artis_model_atomic(m);
  artis_run_params rp;
  artis_model_run_params(m, &rp);
  const int64_t np = artis_model_npts_model(m);
  const int64_t nion = np * at.nelements * at.maxnions;
  std::vector<double> J(np), nuJ(np), ff(np), col(np), gam(nion), bfh(nion), emiss(np);
  std::vector<int32_t> ec(at.nlines), ac(at.nlines);
  std::vector<artis_packet> packets(npkts);
  if (pellets) {
    // read_gamma_spectrum (gammapkt.cc:58-89): line count, then "E[MeV] probability" rows
    const char *files[2] = {"ni56_lines.txt", "co56_lines.txt"};
    for (int nuc = 0; nuc < 2; nuc++) {
      std::ifstream in(std::string(argv[11]) + "/" + files[nuc]);
      int nl = 0;
      if (!(in >> nl) || nl <= 0) {
        std::fprintf(stderr, "cannot read %s\n", files[nuc]);
        return 1;
      }
      std::vector<double> en(nl), pr(nl);
      for (int j = 0; j < nl; j++) in >> en[j] >> pr[j];
      if (artis_model_set_gamma_lines(m, nuc, nl, en.data(), pr.data()) != 0) return 1;
    }
    if (artis_model_init_pellets(m, npkts, seed, 1e45, 0.5 * cfg.tmin_days, 0.02, packets.data()) != 0) return 1;
  } else if (artis_model_init_rpackets(m, nts0, npkts, seed, 1e45, packets.data()) != 0) {
    return 1;
  }

  {
    artis_amd::PacketEngine engine(0, at, *artis_model_geometry(m), rp);
    if (pellets) engine.init_gamma(*artis_model_gamma_spectra(m));
    const char *rccl = std::getenv("ARTIS_DRIVER_RCCL");
    const bool reduced = rccl && rccl[0] == '1';
    if (reduced) {
      unsigned char id[ARTIS_COMM_ID_BYTES];
      artis_amd::PacketEngine::unique_id(id);
      engine.comm_init(0, 1, id);
    }
    int last_nts = -1;
    for (int nts = nts0; nts < nts0 + nsteps && nts < cfg.ntstep; nts++) {
      last_nts = nts;
      artis_amd::check(artis_model_set_timestep(m, nts), "update_grid stand-in");
      engine.upload_cellstate(nts, *artis_model_cellstate(m));
      // zero_estimators (emissivities.cc:138-170)
      artis_estimators est{};
      for (auto *v : {&J, &nuJ, &ff, &col, &gam, &bfh}) std::fill(v->begin(), v->end(), 0.);
      std::fill(ec.begin(), ec.end(), 0);
      std::fill(ac.begin(), ac.end(), 0);
      est.J = J.data();
      est.nuJ = nuJ.data();
      est.ffheatingestimator = ff.data();
      est.colheatingestimator = col.data();
      est.gammaestimator = gam.data();
      est.bfheatingestimator = bfh.data();
      est.ecounter = ec.data();
      est.acounter = ac.data();
      std::fill(emiss.begin(), emiss.end(), 0.);
      est.rpkt_emiss = emiss.data();
      if (reduced)
        engine.update_packets_reduced(rp.rank, nts, packets.data(), npkts, est);
      else
        engine.update_packets(rp.rank, nts, packets.data(), npkts, est);
      double jsum = 0.;
      for (double v : J) jsum += v;
      artis_amd::check(artis_write_temp_packetsfile(outdir.c_str(), nts, rp.rank, packets.data(), npkts),
                       "write_temp_packetsfile");
      std::printf("nts %d nesc %lld cmf_lum %.17g gamma_dep %.17g pellet_decays %lld Jsum %.17g transport_ms %.3f\n",
                  nts, (long long)est.nesc, est.cmf_lum, est.gamma_dep, (long long)est.pellet_decays, jsum,
                  engine.last_transport_ms());
    }
    const char *tev = std::getenv("ARTIS_DRIVER_TE");
    if (tev && tev[0] == '1' && last_nts >= 0) {
      // update_grid for the next timestep: the temperature / ionisation solution from this timestep's estimators
      TeCase c;
      te_from_estimators(at, *artis_model_geometry(m), *artis_model_cellstate(m), *artis_model_te_tables(m), last_nts,
                         (int)np, J, nuJ, ff, col, gam, bfh, c);
      std::ofstream o(outdir + "/te_case.bin", std::ios::binary);
      // inputs (as handed to the engine), then the outputs
      for (const auto *v : {&c.TR, &c.W, &c.TJ, &c.Te, &c.gp}) put(o, *v);
      put(o, c.mgi);
      put(o, c.thick);
      for (const auto *v : {&c.ff, &c.col, &c.gam, &c.bfh, &c.vol}) put(o, *v);
      put(o, c.meanw);
      const double pv[2] = {c.par.t_current, c.par.tmin};
      o.write((const char *)pv, sizeof pv);
      engine.solve_temperatures(*artis_model_te_tables(m), c.par, c.cells);
      for (const auto *v : {&c.Te, &c.gp, &c.nne, &c.nnetot, &c.pf}) put(o, *v);
      for (const auto *v : {&c.totcool, &c.ccion, &c.rates}) put(o, *v);
      put(o, c.iters);
      int rooted = 0;
      for (int k : c.mgi) rooted += c.iters[k] > 0;
      std::printf("te cells %zu rooted %d\n", c.mgi.size(), rooted);
    }
  }
  // the final packet list as the reference writes it at the end of the run (sn3d.cc:640-645)
  artis_amd::check(artis_write_packets((outdir + "/packets00_0000.out").c_str(), packets.data(), npkts),
                   "write_packets");
  artis_model_free(m);
  return 0;
}
