"""The drop-in ABI view used by the shim tests: re-exported from the
package (nav-slam_amd/navslam/abi.py) so bench.py and the tests share it."""
from navslam.abi import KDNode, Point, Pos, Shim, make_types, preorder  # noqa: F401
