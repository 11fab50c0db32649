// Program.cs -- headless Game1 loop (Game1.cs:60-96 without MonoGame): fixed-step Update calls
// on one walker, the ConsoleRenderer.RolloutInformation lines (ConsoleRenderer.cs:51-76) every
// second of simulated time, and the data file at the end.
//   dotnet run -c Release -- [frames] [data-file]
using System;
using NEA.Native;

int frames = args.Length > 0 ? int.Parse(args[0]) : 6000;
string? dataFile = args.Length > 1 ? args[1] : null;
using var env = new HeadlessEnvironment();
float dt = (float)(166667.0 / 10000000.0);  // Game.TargetElapsedTime (fixed step)
for (int f = 0; f < frames; f++)
{
    env.Update(dt);
    if (f % 60 != 59) continue;
    var (episode, step, distance, avg, best, pastAvg, s) = env.GetConsoleInformation();
    Console.WriteLine($"Episode {episode}, timestep {step} ({((float)step / 1000) * 100f} % of max timesteps)");
    Console.WriteLine($"Current average reward: {avg}  Current distance: {distance}");
    Console.WriteLine($"Previous average reward: {pastAvg}  Best distance: {best}");
    Console.WriteLine($"Body position scaled: ({s[0]}, {s[1]})  Body linear velocity: ({s[6]}, {s[7]})");
}
if (dataFile != null) env.CreateDataFile(dataFile);
