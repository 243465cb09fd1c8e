"""MI355X-native stereo visual-odometry front end (drop-in for the per-frame
path of ivario123/r7020e-visual-odometry's VO.m).  See DESIGN.md."""
