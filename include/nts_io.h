/*
 * nts_io.h — the reference's on-disk input formats at scale (libnts_io.so).
 *
 * Host-side C-ABI used by the data loaders (sample-based-gnn_amd/nts/dataloader.py):
 *  - binary edge list of {uint32 src; uint32 dst} pairs (EdgeUnit<Empty>,
 *    core/graph.hpp:1129-1186), memory-mapped and read in caller-sized chunks
 *    so a file beyond host RAM streams to the device;
 *  - text feature / label / mask files parsed in parallel with the reference's
 *    lock-step semantics (GNNDatum::readFeature_Label_Mask,
 *    core/ntsDataloador.hpp:999-1064): the k-th feature line `id f_1 .. f_F`
 *    fills features[id], the k-th label line `id label` gives labels[id], the
 *    k-th mask line `id train|eval|val|test|...` gives masks[id] = 0/1/1/2/3.
 *    Rows of ids that never appear are left as the caller initialised them.
 * Return 0 on success; the message of a failure is nts_io_last_error().
 */
#ifndef NTS_IO_H
#define NTS_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NTS_IO_OK 0
#define NTS_IO_ERR 1

const char *nts_io_last_error(void);
/* |E| of a binary edge file (bytes / 8), or -1 */
int64_t nts_io_edge_count(const char *path);
/* edges [first, first + count) into src[count], dst[count] */
int nts_io_read_edges(const char *path, uint64_t first, uint64_t count, uint32_t *src,
                      uint32_t *dst);
/* features [n_vertices x F] row-major, labels [n_vertices], masks [n_vertices] */
int nts_io_read_feature_label_mask(const char *feature_path, const char *label_path,
                                   const char *mask_path, uint64_t n_vertices, uint32_t F,
                                   float *features, int64_t *labels, int32_t *masks,
                                   int threads);

#ifdef __cplusplus
}
#endif
#endif /* NTS_IO_H */
