// RayTracer.cs -- drop-in replacement for Raytracer/RayTracer.cs's RayTracer class that
// renders through libraytracer_hip (MI355X, gfx950).  Same public surface as the reference
// (RayTracer.cs:437-1062): ctor RayTracer(Surface), `screen`, Tick(), OnKeyPress(e),
// OnMouseMove(e).  template.cs and surface.cs stay untouched.
//
// Build: add this file instead of the reference RayTracer.cs to InfogrRaytracer.csproj
// (net6.0, OpenTK 4.7.1) and put libraytracer_hip.so next to the executable (or on
// LD_LIBRARY_PATH).  Not buildable in the MI355X image (no dotnet); see INTEGRATION.md.
using System.Runtime.InteropServices;
using OpenTK.Windowing.Common;
using OpenTK.Windowing.GraphicsLibraryFramework;

namespace Template;

internal static class Native {
    private const string Lib = "raytracer_hip";
    internal const int AbiVersion = 10;  // RT_ABI_VERSION of the include/raytracer_hip.h these declarations follow

    [StructLayout(LayoutKind.Sequential)] internal struct Vec3 { public float X, Y, Z; public Vec3(float x, float y, float z) { X = x; Y = y; Z = z; } }
    [StructLayout(LayoutKind.Sequential)] internal struct Material { public Vec3 Kd, Ka, Ks; public float N; public Vec3 Km; }
    [StructLayout(LayoutKind.Sequential)] internal struct Sphere { public Vec3 Center; public float Radius; public Material Material; }
    [StructLayout(LayoutKind.Sequential)] internal struct Plane { public Vec3 Center, Normal; public Material Material; }
    [StructLayout(LayoutKind.Sequential)] internal struct Light { public Vec3 Position; public float Intensity; }
    [StructLayout(LayoutKind.Sequential)] internal struct Camera { public Vec3 Position; public float Yaw, Pitch; }

    [DllImport(Lib)] internal static extern int rt_abi_version();
    [DllImport(Lib)] internal static extern int rt_create(int nGpus, out IntPtr ctx);
    [DllImport(Lib)] internal static extern void rt_destroy(IntPtr ctx);
    [DllImport(Lib)] internal static extern IntPtr rt_last_error(IntPtr ctx);
    [DllImport(Lib)] internal static extern int rt_set_scene(IntPtr ctx, Sphere[] s, int ns, Plane[] p, int np,
                                                            Light[] l, int nl, Vec3 ambient, int recursionLimit);
    [DllImport(Lib)] internal static extern int rt_set_camera(IntPtr ctx, ref Camera c);
    [DllImport(Lib)] internal static extern int rt_camera_on_key(ref Camera c, int key);
    [DllImport(Lib)] internal static extern int rt_camera_on_mouse_move(ref Camera c, float dx, float dy);
    [DllImport(Lib)] internal static extern int rt_register_host(IntPtr ctx, IntPtr p, UIntPtr bytes);
    [DllImport(Lib)] internal static extern int rt_unregister_host(IntPtr ctx, IntPtr p);
    [DllImport(Lib)] internal static extern int rt_render(IntPtr ctx, int w, int h, IntPtr pixels);
    // ABI v2+ additions (not needed by the synchronous Tick below): pipelined frames, debug view, timing
    // (ABI 4/5's multi-process and diagnostic pieces -- batched band launches, tile codec, rt_create_ex,
    // rt_count_work -- are declared in INTEGRATION.md)
    [StructLayout(LayoutKind.Sequential)] internal struct Segment { public Vec3 Origin, End; public int Kind, Pixel; }
    [DllImport(Lib)] internal static extern int rt_render_async(IntPtr ctx, int w, int h, IntPtr pixels);
    [DllImport(Lib)] internal static extern int rt_wait(IntPtr ctx);
    [DllImport(Lib)] internal static extern int rt_debug_segments(IntPtr ctx, int w, int h, int stride,
                                                                 [Out] Segment[] segments, int capacity, out int count);
    [DllImport(Lib)] internal static extern int rt_set_timing(IntPtr ctx, int every);
    [DllImport(Lib)] internal static extern int rt_dispatch_order(IntPtr ctx, out int order);
    [DllImport(Lib)] internal static extern int rt_set_counting(IntPtr ctx, int on);  // ABI 10

    internal static void Check(int rc, IntPtr ctx) {
        if (rc != 0) throw new InvalidOperationException($"libraytracer_hip error {rc}: {Marshal.PtrToStringAnsi(rt_last_error(ctx))}");
    }
}

internal sealed class RayTracer : IDisposable {
    public readonly Surface screen;                       // RayTracer.cs:506
    private readonly IntPtr _ctx;
    private GCHandle _pin;
    private Native.Camera _camera;                        // _cameraPosition/_yaw/_pitch, :494-502

    public RayTracer(Surface screen) {                    // RayTracer.cs:535-537
        this.screen = screen;
        // the library must implement the ABI these declarations bind (struct layouts, entry points)
        int abi = Native.rt_abi_version();
        if (abi != Native.AbiVersion)
            throw new InvalidOperationException(
                $"libraytracer_hip ABI {abi}, this binding needs ABI {Native.AbiVersion}: rebuild or update the library");
        int nGpus = int.TryParse(Environment.GetEnvironmentVariable("RT_GPUS"), out int g) ? g : 1;
        Native.Check(Native.rt_create(nGpus, out _ctx), IntPtr.Zero);
        // the reference's Tick counts no rays: the display loop runs without the library's work counters
        Native.Check(Native.rt_set_counting(_ctx, 0), _ctx);
        // the hard-coded scene of RayTracer.cs:441-469
        static Native.Vec3 V(float x, float y, float z) => new(x, y, z);
        static Native.Material M(Native.Vec3 kd, Native.Vec3 ka, Native.Vec3 ks, float n, Native.Vec3 km) =>
            new() { Kd = kd, Ka = ka, Ks = ks, N = n, Km = km };
        var zero = V(0, 0, 0);
        var spheres = new[] {
            new Native.Sphere { Center = V(2.5f, 0, 8), Radius = 1, Material = M(V(1, 0, 0), V(1, 0, 0), zero, 0, zero) },
            new Native.Sphere { Center = V(3, 0, 5), Radius = 1, Material = M(V(0, 1, 0), V(0, 1, 0), V(0.4f, 0.4f, 0.4f), 1, zero) },
            new Native.Sphere { Center = V(-3, 1, 8), Radius = 1, Material = M(zero, zero, zero, 0, V(1, 1, 1)) },
        };
        var planes = new[] {
            new Native.Plane { Center = V(0, -1, 0), Normal = V(0, 1, 0),
                               Material = M(V(1, 1, 1), V(0.5f, 0.5f, 0.5f), V(1, 1, 1), 0.5f, V(1, 1, 1)) },
        };
        var lights = new[] {
            new Native.Light { Position = V(-3, 1, -3), Intensity = 1 },
            new Native.Light { Position = V(33, 1, 10), Intensity = 1 },
        };
        float amb = 43f / 255f;
        Native.Check(Native.rt_set_scene(_ctx, spheres, 3, planes, 1, lights, 2, V(amb, amb, amb), 32), _ctx);
        // pin Surface.pixels once: the library's D2H copy lands directly in the managed array
        _pin = GCHandle.Alloc(screen.pixels, GCHandleType.Pinned);
        Native.Check(Native.rt_register_host(_ctx, _pin.AddrOfPinnedObject(),
                                             (UIntPtr)(screen.pixels.Length * sizeof(int))), _ctx);
    }

    public void Tick() {                                  // RayTracer.cs:886-935
        Native.Check(Native.rt_set_camera(_ctx, ref _camera), _ctx);
        Native.Check(Native.rt_render(_ctx, screen.width, screen.height, _pin.AddrOfPinnedObject()), _ctx);
    }

    public void OnKeyPress(KeyboardKeyEventArgs e) {      // RayTracer.cs:543-554
        int key = e.Key switch {
            Keys.W => 1, Keys.A => 2, Keys.S => 3, Keys.D => 4, Keys.Space => 5,
            Keys.LeftShift or Keys.RightShift => 6, _ => 0
        };
        Native.Check(Native.rt_camera_on_key(ref _camera, key), IntPtr.Zero);
    }

    public void OnMouseMove(MouseMoveEventArgs e) {       // RayTracer.cs:1058-1061
        Native.Check(Native.rt_camera_on_mouse_move(ref _camera, e.DeltaX, e.DeltaY), IntPtr.Zero);
    }

    public void Dispose() {
        if (_pin.IsAllocated) {
            Native.rt_unregister_host(_ctx, _pin.AddrOfPinnedObject());
            _pin.Free();
        }
        Native.rt_destroy(_ctx);
    }
}
