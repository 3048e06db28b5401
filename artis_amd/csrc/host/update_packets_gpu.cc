// update_packets_gpu.cc -- see update_packets_gpu.h
#include "update_packets_gpu.h"

#include <cstdio>
#include <cstdlib>

#include "artis_layout_check.h"

namespace artis_amd {

void check(int rc, const char *what) {
  if (rc != 0) {
    std::fprintf(stderr, "[artis_gpu] %s failed (status %d): %s\n", what, rc, artis_gpu_last_error());
    std::fflush(stderr);
    std::abort();
  }
}

PacketEngine::PacketEngine(int device, const artis_atomic_tables &atomic, const artis_geometry &geometry,
                           const artis_run_params &params) {
  check(artis_gpu_abi_version() == ARTIS_GPU_ABI_VERSION ? 0 : ARTIS_ERR_BAD_ARGUMENT, "artis_gpu_abi_version");
  check(artis_gpu_init(device, &atomic, &geometry, &params), "artis_gpu_init");
}

PacketEngine::~PacketEngine() { artis_gpu_finalize(); }

void PacketEngine::init_gamma(const artis_gamma_spectra &spectra) {
  check(artis_gpu_init_gamma(&spectra), "artis_gpu_init_gamma");
}

void PacketEngine::upload_cellstate(int nts, const artis_cell_state &cells) {
  check(artis_gpu_upload_cellstate(nts, &cells), "artis_gpu_upload_cellstate");
}

void PacketEngine::solve_temperatures(const artis_te_tables &tables, const artis_te_params &params,
                                      artis_te_cells &cells) {
  check(artis_gpu_solve_temperatures(&tables, &params, &cells), "artis_gpu_solve_temperatures");
}

void PacketEngine::update_grid_nlte(const artis_nt_shells *shells, const artis_nlte_params &params,
                                    artis_nlte_cells &cells) {
  check(artis_gpu_update_grid_nlte(shells, &params, &cells), "artis_gpu_update_grid_nlte");
}

void PacketEngine::prepare_temperatures(const artis_te_tables &tables, const artis_te_params &params,
                                        const artis_ug_prepare &prep, const artis_te_cells &cells) {
  check(artis_gpu_prepare_temperatures(&tables, &params, &prep, &cells), "artis_gpu_prepare_temperatures");
}

void PacketEngine::update_packets(int my_rank, int nts, artis_packet *packets, int npkts, artis_estimators &est) {
  check(artis_gpu_update_packets(my_rank, nts, packets, npkts, &est), "artis_gpu_update_packets");
}

void PacketEngine::unique_id(unsigned char id[ARTIS_COMM_ID_BYTES]) {
  check(artis_gpu_comm_unique_id(id), "artis_gpu_comm_unique_id");
}

void PacketEngine::comm_init(int rank, int nranks, const unsigned char id[ARTIS_COMM_ID_BYTES]) {
  check(artis_gpu_comm_init(rank, nranks, id), "artis_gpu_comm_init");
}

void PacketEngine::update_packets_reduced(int my_rank, int nts, artis_packet *packets, int npkts,
                                          artis_estimators &est) {
  check(artis_gpu_packets_upload(packets, npkts), "artis_gpu_packets_upload");
  check(artis_gpu_estimators_zero(), "artis_gpu_estimators_zero");
  check(artis_gpu_update_packets_resident(my_rank, nts), "artis_gpu_update_packets_resident");
  check(artis_gpu_estimators_allreduce(), "artis_gpu_estimators_allreduce");
  check(artis_gpu_packets_download(packets, npkts), "artis_gpu_packets_download");
  check(artis_gpu_estimators_download(&est), "artis_gpu_estimators_download");
}

double PacketEngine::last_transport_ms() const { return artis_gpu_last_transport_ms(); }

}  // namespace artis_amd
