"""dbscan_amd -- MI355X-native (gfx950) local DBSCAN fit for dbscan-on-spark.

Drop-in for the reference's hot path `new LocalDBSCANNaive(eps, minPoints).fit(points)`
(DBSCAN.scala:153-154).  Compute lives in libdbscan_hip.so (hand-written HIP kernels, C-ABI
in include/dbscan_hip.h); this package is the host-side mirror of the reference interface.
"""
from ._lib import (DBSCANError, Handle, MODE_ARCHERY, MODE_ARCHERY_F32BOX, MODE_NAIVE, LIB_PATH, load)  # noqa: F401
from .local import (DBSCANLabeledPoint, DBSCANPoint, Flag, LocalDBSCANArchery,  # noqa: F401
                    LocalDBSCANNaive, Unknown, duplicate, fit_arrays, fit_batch, train_node)
from .partition import DBSCANRectangle, EvenSplitPartitioner  # noqa: F401
from .train import DBSCAN  # noqa: F401
