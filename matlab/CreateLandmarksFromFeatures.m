function landmarks = CreateLandmarksFromFeatures(features_l, features_r, intrinsics_l, intrinsics_r, pose, current_landmarks)
%CREATELANDMARKSFROMFEATURES libvo (MI355X) shadow of the reference's own function.
%   Same signature and result as reference CreateLandmarksFromFeatures.m:1-21:
%   odd rows only, z in [0, 80], zero rows kept (at least 2 rows), world =
%   pose.transformPointsForward, appended to current_landmarks.  VO.m:160
%   passes points VO.m:145-158 has already filtered, so the device's own
%   new-landmark filter runs against no old points.  intrinsics_l/_r are the
%   3 x 4 camera matrices p1, p2 (VO.m:27-32), as in the reference.
    rows = vo_mex('landmarks', features_l, features_r, double(intrinsics_l), double(intrinsics_r), pose.A);
    landmarks = [current_landmarks; rows];
end
