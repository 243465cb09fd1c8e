function desc = vo_sift_cache(op, I, loc, d)
%VO_SIFT_CACHE descriptors of the last few libvo detections, keyed by image and locations
%   (VO.m detects the left and the right image before it extracts either, VO.m:79-84).
    persistent entries
    desc = [];
    switch op
        case 'put'
            e = struct('I', I, 'loc', loc, 'desc', d);
            if isempty(entries)
                entries = e;
            else
                entries = [e, entries(1:min(end, 3))];
            end
        case 'get'
            for k = 1:numel(entries)
                if isequal(entries(k).loc, loc) && isequal(entries(k).I, I)
                    desc = entries(k).desc;
                    return;
                end
            end
        case 'clear'
            entries = [];
    end
end
