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
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "artis_io.h"
#include "artis_layout_check.h"
#include "model_synth.h"
#include "update_packets_gpu.h"

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
    for (int nts = nts0; nts < nts0 + nsteps && nts < cfg.ntstep; nts++) {
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
  }
  // the final packet list as the reference writes it at the end of the run (sn3d.cc:640-645)
  artis_amd::check(artis_write_packets((outdir + "/packets00_0000.out").c_str(), packets.data(), npkts),
                   "write_packets");
  artis_model_free(m);
  return 0;
}
