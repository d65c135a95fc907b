"""navslam — MI355X-native scan-matching front end for NAV-SLAM (host side)."""
