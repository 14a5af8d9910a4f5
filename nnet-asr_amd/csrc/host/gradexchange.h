// gradexchange.h -- data-parallel gradient exchange interface used by CuNetwork::TrainBunch.
//
// The reference has no multi-GPU path; its CPU Platform sums per-thread
// gradients row-slice by row-slice into a shared accumulator (src/TNetLib/Platform.h:307-335,
// BiasedLinearity.cc:90-178).  On MI355X the same "sum of the ranks' gradients, then one identical
// update everywhere" is an RCCL all-reduce over xGMI, issued per layer as soon as that layer's
// gradient exists, on a communication stream, so it overlaps the backward GEMMs of the layers
// below (rccl_exchange.cpp).
#pragma once

#include <cstddef>

namespace TNet {

class CuUpdatableComponent;

class GradExchange {
 public:
  virtual ~GradExchange() {}
  virtual int Rank() const = 0;
  virtual int WorldSize() const = 0;
  /// Called after comp.ComputeGradient() was enqueued on the compute stream: start reducing
  /// comp.GradientBlocks() asynchronously.
  virtual void Submit(CuUpdatableComponent& comp) = 0;
  /// Make the compute stream wait until every submitted reduction has finished.
  virtual void WaitAll() = 0;
  /// Frames of the global bunch (sum over ranks) for the GRADDIVFRM normalisation.
  virtual size_t GlobalRows(size_t local_rows) = 0;
  /// Sum small host statistics over ranks (epoch-end MergeStats); blocking.
  virtual void AllReduceHost(double* v, int n) = 0;
};

}  // namespace TNet
