"""MI355X-native MR-HDBSCAN* hot path (drop-in for the reference's hdbscanstar / distance /
databubbles / mappers / reducers operators), backed by the HIP library libhdbmi.so.

See DESIGN.md.  Import via importlib (the directory name is not an identifier):
    pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
"""
from . import _capi
from ._capi import (BUBBLE_CF, BUBBLE_COMBINESTEP, CORE_EXCL_SELF, CORE_INCL_SELF,
                    CORE_INCL_SELF_CUMULATIVE, JMAX, ArithmeticException,
                    ArrayIndexOutOfBoundsException, Context, HdbError, IllegalStateException,
                    NullPointerException, NumberFormatException, lib)
from .databubbles import (CombineStep, FirstStep, HdbscanDataBubbles, LocalModelReduceByKey,
                          bubble_stats, merge_sorted_runs, nearest_sample, sort_edges_desc)
from .driver import MRHDBSCANStar
from .formats import (MapperDataset_github, double_to_string, format_local_mst, parse_local_mst,
                      read_dataset)
from .hdbscanstar import (CosineSimilarity, DistanceCalculator, EuclideanDistance, HDBSCANStar,
                          ManhattanDistance, PearsonCorrelation, SupremumDistance, UndirectedGraph,
                          distance_rows, flat_labels)

__all__ = [n for n in dir() if not n.startswith("_")]
