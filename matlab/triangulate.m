function worldPoints = triangulate(matchedPoints1, matchedPoints2, cameraMatrix1, cameraMatrix2)
%TRIANGULATE libvo (MI355X) shadow: worldPoints = triangulate(x1, x2, P1, P2)
%   reference call sites: VO.m:113-116, CreateLandmarksFromFeatures.m:7.
%   x1, x2: N x 2 points (or point objects), P1, P2: 3 x 4 camera matrices
%   (VO.m:27-32).  Linear DLT per point in double, result returned as single
%   (VO.m passes single Locations).
    if isobject(matchedPoints1), matchedPoints1 = matchedPoints1.Location; end
    if isobject(matchedPoints2), matchedPoints2 = matchedPoints2.Location; end
    worldPoints = vo_mex('triangulate', matchedPoints1, matchedPoints2, double(cameraMatrix1), double(cameraMatrix2));
end
