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
// ARTIS_DRIVER_TE=1: after the last timestep, update_grid's estimator preparation and temperature / ionisation
// solution on the GPU (PacketEngine::prepare_temperatures + solve_temperatures) from that timestep's own raw
// estimators; inputs and outputs go to <outdir>/te_case.bin for the oracle replay in tests/test_host_driver.py.
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
// update_grid for the timestep after the run's last one, on the GPU: the cells' previous state (the model's cell
// state), the run's raw estimators, artis_gpu_prepare_temperatures (update_grid.cc:1041-1150) and then
// artis_gpu_solve_temperatures.  Stand-ins where the reference needs data this synthetic model does not carry:
// mean atomic weight 2.1 Z m_H, vol_init from the uniform grid's cell count per model cell.
struct TeCase {
  std::vector<int32_t> mgi;
  std::vector<float> TR, W, TJ, rho, abund, meanw, Te, gp, nne, nnetot, pf, nne_old, pf_old, TR_new, W_new, TJ_new;
  std::vector<int16_t> thick;
  std::vector<double> vol, ff, col, gam, bfh, totcool, ccion, rates, renorm;
  std::vector<int32_t> iters;
  artis_te_cells cells{};
  artis_te_params par{};
  artis_ug_prepare prep{};
};
void te_setup(const artis_atomic_tables &at, const artis_geometry &g, const artis_cell_state &cs, int nts_next, int nts,
              int np, const std::vector<double> &J, const std::vector<double> &nuJ, const std::vector<double> &ff,
              const std::vector<double> &col, const std::vector<double> &gam, const std::vector<double> &bfh,
              TeCase &c) {
  const int nel = at.nelements, ni = at.nions_total, mx = at.maxnions;
  const double MH = 1.67352e-24;
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
  c.nne_old.assign(cs.nne, cs.nne + np);
  c.pf_old.assign(cs.partfunct, cs.partfunct + (size_t)np * ni);
  c.meanw.resize((size_t)np * nel);
  c.vol.resize(np);
  for (int mgi = 0; mgi < np; mgi++) {
    for (int e = 0; e < nel; e++) c.meanw[(size_t)mgi * nel + e] = (float)(2.1 * at.elem_anumber[e] * MH);
    c.vol[mgi] = wid * wid * wid * count[mgi];
    if (c.rho[mgi] > 0 && count[mgi] > 0) c.mgi.push_back(mgi);
  }
  c.TR_new.assign(np, 0.f);
  c.W_new.assign(np, 0.f);
  c.TJ_new.assign(np, 0.f);
  c.ff.assign(np, 0.);
  c.col.assign(np, 0.);
  c.gam.assign((size_t)np * nel * mx, 0.);
  c.bfh.assign((size_t)np * nel * mx, 0.);
  c.renorm.assign((size_t)np * nel * mx, 0.);
  c.nne.assign(np, 0.f);
  c.nnetot.assign(np, 0.f);
  c.pf.assign((size_t)np * ni, 0.f);
  c.totcool.assign(np, 0.);
  c.ccion.assign((size_t)np * ni, 0.);
  c.rates.assign((size_t)np * ARTIS_TE_NRATES, 0.);
  c.iters.assign(np, 0);
  artis_ug_prepare &p = c.prep;
  p.deltat = g.ts_width[nts];                // time_step[nts_prev].width (update_grid.cc:1316)
  p.tratmid = g.ts_mid[nts_next] / g.tmin;   // time_step[nts].mid / tmin of the timestep being prepared
  p.nprocs = 1;
  p.J = J.data();
  p.nuJ = nuJ.data();
  p.ffheating = ff.data();
  p.colheating = col.data();
  p.gammaestimator = gam.data();
  p.bfheatingestimator = bfh.data();
  p.nne = c.nne_old.data();
  p.partfunct = c.pf_old.data();
  p.TR_out = c.TR_new.data();
  p.W_out = c.W_new.data();
  p.TJ_out = c.TJ_new.data();
  p.ffheating_out = c.ff.data();
  p.colheating_out = c.col.data();
  p.gamma_out = c.gam.data();
  p.bfheating_out = c.bfh.data();
  p.corrphotoionrenorm_out = c.renorm.data();
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
  c.par.t_current = g.ts_mid[nts];  // nts_for_te = nts - 1 at titer 0 (update_grid.cc:804)
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
    if (tev && tev[0] == '1' && last_nts >= 0 && last_nts + 1 >= cfg.ntstep) {
      // there is no next timestep to prepare: the reference's update_grid pairs nts with nts_prev = nts - 1
      std::printf("te skipped: the run ended at the last timestep %d\n", last_nts);
    } else if (tev && tev[0] == '1' && last_nts >= 0) {
      // update_grid for the next timestep on the GPU (nts = last_nts + 1, nts_prev = last_nts, as update_grid.cc:1316
      // pairs them): estimator preparation, then the temperature solution
      TeCase c;
      const int nts_next = last_nts + 1;
      te_setup(at, *artis_model_geometry(m), *artis_model_cellstate(m), nts_next, last_nts, (int)np, J, nuJ, ff, col,
               gam, bfh, c);
      std::ofstream o(outdir + "/te_case.bin", std::ios::binary);
      // inputs: the previous state, the raw estimators, the parameters; then the outputs
      for (const auto *v : {&c.TR, &c.W, &c.TJ, &c.Te, &c.gp, &c.nne_old, &c.pf_old}) put(o, *v);
      put(o, c.mgi);
      put(o, c.thick);
      for (const auto *v : {&J, &nuJ, &ff, &col, &gam, &bfh, &c.vol}) put(o, *v);
      put(o, c.meanw);
      const double pv[4] = {c.par.t_current, c.par.tmin, c.prep.deltat, c.prep.tratmid};
      o.write((const char *)pv, sizeof pv);
      const artis_te_tables &tab = *artis_model_te_tables(m);
      engine.prepare_temperatures(tab, c.par, c.prep, c.cells);
      for (const auto *v : {&c.TR_new, &c.W_new, &c.TJ_new}) put(o, *v);
      // the solution reads the prepared radiation field (the estimator inputs already point at the prepared arrays)
      c.cells.TR = c.TR_new.data();
      c.cells.W = c.W_new.data();
      c.cells.TJ = c.TJ_new.data();
      engine.solve_temperatures(tab, c.par, c.cells);
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
