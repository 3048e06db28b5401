// update_packets_gpu.h -- C++ host side of the drop-in: the reference's update_packets interface
// (update_packets.h:6, called at sn3d.cc:574) on top of the C ABI of include/artis_gpu.h.
//
// A reference build links this file and libartis_gpu.so and replaces its update_packets call as shown in
// INTEGRATION.md.  The error behaviour is the reference's: any failure is printed and the process aborts
// (assert_always, sn3d.h:17-29); nothing falls back to a CPU path.
#ifndef ARTIS_UPDATE_PACKETS_GPU_H
#define ARTIS_UPDATE_PACKETS_GPU_H

#include "artis_gpu.h"

namespace artis_amd {

// abort with the engine's message if rc != 0 (reference assert_always semantics)
void check(int rc, const char *what);

// One GPU's engine for the run: owns the device tables; the caller owns packets and estimator arrays.
class PacketEngine {
 public:
  PacketEngine(int device, const artis_atomic_tables &atomic, const artis_geometry &geometry,
               const artis_run_params &params);
  ~PacketEngine();
  PacketEngine(const PacketEngine &) = delete;
  PacketEngine &operator=(const PacketEngine &) = delete;

  // gamma-ray line spectra for pellet decays (gammapkt::init_gamma_linelist, gammapkt.cc:194; called from input())
  void init_gamma(const artis_gamma_spectra &spectra);

  // after update_grid (update_grid.cc:1270) for timestep nts
  void upload_cellstate(int nts, const artis_cell_state &cells);

  // reference update_packets(my_rank, nts, packets) with the packet count and the estimator arrays (globals::
  // and radfield:: in the reference) made explicit; estimators are accumulated, as the reference's are
  void update_packets(int my_rank, int nts, artis_packet *packets, int npkts, artis_estimators &est);

  // Multi-GPU (one process per GPU): join the RCCL communicator of all ranks.  Rank 0 makes the id with
  // unique_id(); the host distributes it (MPI_Bcast in sn3d).
  static void unique_id(unsigned char id[ARTIS_COMM_ID_BYTES]);
  void comm_init(int rank, int nranks, const unsigned char id[ARTIS_COMM_ID_BYTES]);

  // update_packets followed by the reference's mpi_reduce_estimators (sn3d.cc:316-377, radfield.cc:1502-1564)
  // done in HBM: the packed estimator block is all-reduced over RCCL before it is copied into est, so every rank
  // receives the summed estimators (which it would otherwise get from MPI_Allreduce of its host arrays)
  void update_packets_reduced(int my_rank, int nts, artis_packet *packets, int npkts, artis_estimators &est);

  // update_grid's per-cell temperature / ionisation solution for the LTE-population options (the reference's
  // solve_Te_nltepops / LTE branch + calculate_cooling_rates, update_grid.cc:1104-1158, 1199-1205) for the cells in
  // `cells.mgi`, after the host normalised the estimators (update_grid.cc:1041-1150); results written into `cells`
  void solve_temperatures(const artis_te_tables &tables, const artis_te_params &params, artis_te_cells &cells);
  // the estimator preparation before it (update_grid.cc:1041-1150): raw accumulators -> the inputs of
  // solve_temperatures, written to prep's *_out arrays
  void prepare_temperatures(const artis_te_tables &tables, const artis_te_params &params, const artis_ug_prepare &prep,
                            const artis_te_cells &cells);
  // update_grid for the nebular options (artis_gpu_update_grid_nlte: update_grid.cc:1012-1205 with
  // solve_Te_nltepops, nltepop.cc, nonthermal.cc's Spencer-Fano solution), cells in place
  void update_grid_nlte(const artis_nt_shells *shells, const artis_nlte_params &params, artis_nlte_cells &cells);

  double last_transport_ms() const;
};

}  // namespace artis_amd

#endif
